"""Shard-boundary checkpoint / resume (``--resume_dir``).

The reference has no runtime checkpointing: a crash loses the whole pass,
and its only "resume" is the ``<prompts>_updated.pkl`` file that lets a later
run continue *generation* (``/root/reference/main.py:93-94``); disk-mode
``.npy`` spills are deleted as they are consumed (``utils.py:198-204``).

Here a single-GPU or data-parallel run can persist, every ``every`` shards,
the activations that leave the last layer of a shard (one ``.npy`` per
micro-batch, the same format as disk spills) plus a manifest.  A restarted run
with the same inputs finds the newest complete checkpoint whose fingerprint
(model config, plan parameters, token ids) matches and starts at that shard;
everything before it is skipped.  Data-parallel ranks agree on a shard that
all of them hold, so the per-shard weight all-gathers stay matched.  The last
two complete checkpoints are kept (ranks can be at most one apart when one
dies), and the directory is removed when the run completes.

Layout: ``<root>/rank<r>/step<k>/{manifest.json, mb<b>.npy}``, written into
``step<k>.tmp`` and renamed, so a crash mid-write never leaves a manifest
pointing at partial files.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
from typing import Dict, List, Sequence

import numpy as np
import torch

KEEP = 2


def run_fingerprint(cfg, token_seqs: Sequence[Sequence[int]], **params) -> str:
    """Stable hash of everything that determines the inter-shard activations."""
    h = hashlib.sha256()
    h.update(json.dumps(cfg.__dict__, sort_keys=True, default=str).encode())
    h.update(json.dumps(params, sort_keys=True, default=str).encode())
    for s in token_seqs:
        h.update(np.asarray(s, dtype=np.int64).tobytes())
        h.update(b"|")
    return h.hexdigest()


class RunCheckpoint:
    def __init__(self, root: str, fingerprint: str, rank: int = 0):
        self.root = root
        self.dir = os.path.join(root, f"rank{rank}")
        self.fingerprint = fingerprint
        os.makedirs(self.dir, exist_ok=True)

    def _step_dir(self, k: int, tmp: bool = False) -> str:
        return os.path.join(self.dir, f"step{k}" + (".tmp" if tmp else ""))

    def available(self) -> List[int]:
        """Next-shard indices of complete checkpoints made by this exact run."""
        out = []
        for name in os.listdir(self.dir):
            if not name.startswith("step") or name.endswith(".tmp"):
                continue
            try:
                with open(os.path.join(self.dir, name, "manifest.json")) as f:
                    man = json.load(f)
            except (OSError, ValueError):
                continue
            if man.get("fingerprint") == self.fingerprint:
                out.append(int(man["next_shard"]))
        return sorted(out)

    def save_state(self, next_shard: int, key: int, t: torch.Tensor) -> None:
        d = self._step_dir(next_shard, tmp=True)
        os.makedirs(d, exist_ok=True)
        a = t.detach().cpu()
        arr = a.view(torch.int16).numpy().view(np.uint16) if a.dtype == torch.bfloat16 else a.numpy()
        np.save(os.path.join(d, f"mb{key}.npy"), arr)

    def commit(self, next_shard: int, keys: Sequence[int], dtype: torch.dtype) -> None:
        tmp, final = self._step_dir(next_shard, tmp=True), self._step_dir(next_shard)
        os.makedirs(tmp, exist_ok=True)        # (a data-parallel rank without prompts commits no state)
        missing = [k for k in keys if not os.path.exists(os.path.join(tmp, f"mb{k}.npy"))]
        if missing:
            raise RuntimeError(f"checkpoint step{next_shard}: states missing for micro-batches {missing}")
        with open(os.path.join(tmp, "manifest.json"), "w") as f:
            json.dump({"fingerprint": self.fingerprint, "next_shard": next_shard, "keys": list(keys),
                       "dtype": str(dtype)}, f)
        if os.path.exists(final):
            shutil.rmtree(final)
        os.replace(tmp, final)
        for k in self.available()[:-KEEP]:
            shutil.rmtree(self._step_dir(k), ignore_errors=True)

    def load(self, next_shard: int) -> Dict[int, torch.Tensor]:
        d = self._step_dir(next_shard)
        with open(os.path.join(d, "manifest.json")) as f:
            man = json.load(f)
        bf16 = man["dtype"] == str(torch.bfloat16)
        out = {}
        for k in man["keys"]:
            arr = np.load(os.path.join(d, f"mb{k}.npy"))
            t = torch.from_numpy(arr)
            out[int(k)] = t.view(torch.bfloat16) if bf16 else t
        return out

    def clear(self) -> None:
        shutil.rmtree(self.dir, ignore_errors=True)
        try:
            os.rmdir(self.root)
        except OSError:
            pass
