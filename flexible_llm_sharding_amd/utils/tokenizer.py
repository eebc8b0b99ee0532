"""Tokenization contract and a deterministic synthetic tokenizer.

Reference contract (``/root/reference/utils.py:102-104, 246-258``):

* the tokenizer is loaded from ``model_path``; ``pad_token = eos_token``,
  ``padding_side = "right"``;
* prefix  -> ``tok(prefix, truncation=True, max_length=4096).input_ids`` (BOS kept);
* suffixes -> ``tok(list(suffixes), padding=True, truncation=True,
  max_length=4096).input_ids[:, 1:]`` (BOS dropped, right padded with EOS);
* ``suffix_eos = (suffix != pad).sum(1) - 1`` — the position whose next-token
  distribution is scored.

No tokenizer assets can be downloaded in this environment, so
:func:`write_synthetic_tokenizer` writes a genuine HF ``tokenizer.json`` (a
WordLevel vocabulary of ``vocab_size`` pseudo-words with a ``<s> $A``
template) that ``AutoTokenizer.from_pretrained`` loads exactly like a real
Llama tokenizer directory.
"""
from __future__ import annotations

import json
import os
import string
import weakref
from dataclasses import dataclass
from typing import List, Sequence, Tuple

from ..config import MAX_TOKEN_LEN

_LETTERS = string.ascii_lowercase


def synthetic_word(i: int) -> str:
    """Deterministic pseudo-word for token id ``i`` (ids >= 3)."""
    n = i
    s = ""
    while True:
        s = _LETTERS[n % 26] + s
        n //= 26
        if n == 0:
            break
    return "w" + s


def write_synthetic_tokenizer(model_path: str, vocab_size: int = 32000) -> None:
    from tokenizers import Tokenizer, models, pre_tokenizers, processors, decoders
    from transformers import PreTrainedTokenizerFast

    vocab = {"<unk>": 0, "<s>": 1, "</s>": 2}
    for i in range(3, vocab_size):
        vocab[synthetic_word(i)] = i
    tk = Tokenizer(models.WordLevel(vocab=vocab, unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.WhitespaceSplit()
    tk.post_processor = processors.TemplateProcessing(
        single="<s> $A", pair="<s> $A $B", special_tokens=[("<s>", 1)])
    tk.decoder = decoders.WordPiece(prefix="##", cleanup=False)
    fast = PreTrainedTokenizerFast(tokenizer_object=tk, bos_token="<s>", eos_token="</s>",
                                   unk_token="<unk>", model_max_length=MAX_TOKEN_LEN)
    os.makedirs(model_path, exist_ok=True)
    fast.save_pretrained(model_path)


def load_tokenizer(model_path: str):
    """AutoTokenizer with the reference's pad/padding settings (utils.py:102-104)."""
    from transformers import AutoTokenizer, PreTrainedTokenizerFast
    cls_name = None
    try:
        with open(os.path.join(model_path, "tokenizer_config.json")) as f:
            cls_name = json.load(f).get("tokenizer_class")
    except (OSError, ValueError):
        pass
    if cls_name in ("PreTrainedTokenizerFast", "TokenizersBackend"):
        # an explicit generic fast tokenizer (e.g. ours): do not let AutoTokenizer substitute the
        # model_type's own class from config.json
        tok = PreTrainedTokenizerFast.from_pretrained(model_path)
    else:
        tok = AutoTokenizer.from_pretrained(model_path)
    tok.pad_token = tok.eos_token
    tok.padding_side = "right"
    return tok


@dataclass
class TokenizedPrompt:
    prefix: List[int]                 # [Lp] incl. BOS
    suffixes: List[List[int]]         # n_s rows of real tokens (up to and incl. scored pos)
    padded_len: int                   # Ls of the padded suffix batch (reference shape)
    eos_index: List[int]              # reference suffix_eos (may be -1 -> last column)

    @property
    def n_suffix(self) -> int:
        return len(self.suffixes)

    @property
    def num_tokens(self) -> int:
        return len(self.prefix) + sum(len(s) for s in self.suffixes)

    @property
    def padded_tokens(self) -> int:
        """Tokens the reference computes (prefix + n_s * Ls)."""
        return len(self.prefix) + self.n_suffix * self.padded_len


def tokenize_prompt(tok, prefix: str, suffixes: Sequence[str],
                    max_len: int = MAX_TOKEN_LEN) -> TokenizedPrompt:
    p = tok(prefix, return_attention_mask=False, truncation=True, max_length=max_len)["input_ids"]
    s = tok(list(suffixes), return_attention_mask=False, truncation=True, max_length=max_len,
            padding=True)["input_ids"]
    return _assemble(p, s, tok.pad_token_id)


def _assemble(p, s, pad) -> TokenizedPrompt:
    """prefix ids + the right-padded suffix batch -> TokenizedPrompt (utils.py:250-259)."""
    rows = [list(r[1:]) for r in s]
    Ls = len(rows[0]) if rows else 0
    eos, real = [], []
    for r in rows:
        e = len(r) - r.count(pad) - 1         # (suffix != pad).sum(1) - 1
        eos.append(e)
        idx = e if e >= 0 else Ls - 1     # torch index -1 == last column (reference quirk)
        if idx < 0:
            raise ValueError("empty suffix batch (Ls == 0) cannot be scored")
        # tokens after the scored position cannot influence it (causal): drop them.
        real.append(r[:idx + 1])
    return TokenizedPrompt(list(p), real, Ls, eos)


# prefix string -> ids, per tokenizer: a generation step re-tokenizes the same prefixes (only the
# suffixes grow), and the prefixes are ~70% of the tokenizer's time (32 x 1k tokens: ~4.5 ms of a
# ~65 ms 70B step with suffix K/V reuse).  Tokenization is a pure function of the string.
_PREFIX_IDS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()
_PREFIX_IDS_MAX = 4096


def clear_prefix_ids() -> None:
    """Forget every cached prefix tokenization (benchmarks: each timed call then tokenizes its
    prefixes like a fresh ``main.py`` call, ``/root/reference/utils.py:246-259``)."""
    _PREFIX_IDS.clear()


def _prefix_ids(tok, prefixes: Sequence[str], max_len: int):
    try:
        cache = _PREFIX_IDS.setdefault(tok, {})
    except TypeError:                       # a tokenizer that cannot be weakly referenced
        cache = {}
    miss = sorted({p for p in prefixes if (p, max_len) not in cache})
    if miss:
        if len(cache) + len(miss) > _PREFIX_IDS_MAX:
            cache.clear()
        enc = tok(miss, return_attention_mask=False, truncation=True, max_length=max_len)["input_ids"]
        for p, ids in zip(miss, enc):
            cache[(p, max_len)] = list(ids)
    return [cache[(p, max_len)] for p in prefixes]


def tokenize_prompts(tok, prompts: Sequence[Tuple[str, Sequence[str]]],
                     max_len: int = MAX_TOKEN_LEN) -> List[TokenizedPrompt]:
    """All prompts in two batched tokenizer calls (the fast tokenizer encodes a batch on
    all cores; per-prompt calls cost ~75 ms per 32 x 1k-token prompts, inside every pass);
    prefixes seen before come from a per-tokenizer cache.
    Each prompt's suffix batch is then right-padded to its own longest suffix exactly as
    ``tok(suffixes, padding=True)`` does, so the result equals :func:`tokenize_prompt`."""
    if not prompts:
        return []
    pre = _prefix_ids(tok, [p for p, _ in prompts], max_len)
    flat = [x for _, sufs in prompts for x in sufs]
    enc = tok(flat, return_attention_mask=False, truncation=True, max_length=max_len)["input_ids"] if flat else []
    pad = tok.pad_token_id
    right = getattr(tok, "padding_side", "right") == "right"
    out, j = [], 0
    for (p, sufs), ids in zip(prompts, pre):
        rows = enc[j:j + len(sufs)]
        j += len(sufs)
        L = max((len(r) for r in rows), default=0)
        padded = [list(r) + [pad] * (L - len(r)) if right else [pad] * (L - len(r)) + list(r) for r in rows]
        out.append(_assemble(ids, padded, pad))
    return out
