"""Code-generation invariants of the hand-scheduled GEMM main loops (CPU-only: hipcc cross-compiles
gfx950 here).

The v10 / v11 main loops accumulate with inline-asm MFMAs (common.h / gemm_v11.hip), which hipcc
treats as opaque: if the register allocator ever inserts a copy (v_mov / v_accvgpr_*) of an
accumulator inside the loop, that copy can read an MFMA result before the MFMA has written it
(hipcc pads no hazard inside or right after an asm statement; cdna_hip_programming.md §5.7 item 2).
A first v11 build did exactly that (accumulator <-> fragment register swaps at the loop back-edge:
stale values in the last row group), caught by the GPU bitwise test; this test pins the invariant
at build time for every epilogue instantiation."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


def _asm(src, tmp):
    out = os.path.join(tmp, os.path.basename(src) + ".s")
    cmd = [HIPCC, "--offload-arch=gfx950", "--cuda-device-only", "-S", "-O3", "-std=c++17", "-ffp-contract=fast",
           "-munsafe-fp-atomics", "-I", os.path.join(ROOT, "csrc", "include"), "-I",
           os.path.join(ROOT, "csrc", "kernels"), src, "-o", out]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    return open(out).read().split("\n")


def _main_loops(lines, kernel_re, min_mfma=100):
    """(kernel name, loop body lines) of every loop with >= min_mfma MFMAs in the matching kernels."""
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + kernel_re + r"\S*:", l)]
    ends = [next((j for j in range(s + 1, len(lines)) if lines[j].startswith(".Lfunc_end")), len(lines)) for s in starts]
    for s, e in zip(starts, ends):
        k = lines[s:e]
        for h, l in enumerate(k):
            if "Loop Header" not in l:
                continue
            lab_line = l if l.startswith(".LBB") else k[h - 1]
            if not lab_line.startswith(".LBB"):
                continue
            lab = lab_line.split(":")[0].strip()
            be = [i for i in range(h, len(k)) if re.match(r"\s*s_cbranch_\w+ " + re.escape(lab) + r"\s*$", k[i])]
            if not be:
                continue
            body = k[h:be[0] + 1]
            if sum("v_mfma" in x for x in body) >= min_mfma:
                yield k[0].split(":")[0], body


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("src,kernel,mfmas", [("gemm_v11.hip", "gemm_nt_v11", 384), ("gemm.hip", "gemm_nt_v10", 256)])
def test_gemm_main_loop_has_no_register_copies(tmp_path, src, kernel, mfmas):
    lines = _asm(os.path.join(ROOT, "csrc", "kernels", src), str(tmp_path))
    loops = list(_main_loops(lines, kernel))
    assert loops, f"no main loop found in {kernel}"
    for name, body in loops:
        n_mfma = sum("v_mfma" in x for x in body)
        assert n_mfma == mfmas, (name, n_mfma)
        copies = [x.strip() for x in body if re.search(r"\bv_mov|\bv_accvgpr|\bv_pk_mov", x)]
        assert not copies, (name, copies[:8])


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_skinny_gemm_loop_has_no_register_copies(tmp_path):
    """gemm_nt_skinny<RS, EPI, BN> (gemm_skinny.h): one K-tile per iteration, 2 K-steps x RS row
    subtiles x BN / 64 weight subtiles of asm MFMAs into pinned AGPR accumulators; no copy of any
    register in the loop (a compiled-MFMA build rotated the accumulators through AGPR copies every
    K-tile) and no scratch."""
    lines = _asm(os.path.join(ROOT, "csrc", "kernels", "gemm.hip"), str(tmp_path))
    loops = list(_main_loops(lines, "gemm_nt_skinny", min_mfma=8))
    names = {n for n, _ in loops}
    # (BN 128: RS 2..16 even, BN 256: RS 2..10 even) x NONE / RESID / SWIGLU / F32
    assert len(names) == 4 * (8 + 5), sorted(names)
    for name, body in loops:
        rs, bn = map(int, re.search(r"gemm_nt_skinnyILi(\d+)ELin?\d+ELi(\d+)E", name).groups())
        assert sum("v_mfma" in x for x in body) == rs * bn // 32, name
        copies = [x.strip() for x in body if re.search(r"\bv_mov|\bv_accvgpr|\bv_pk_mov|scratch_", x)]
        assert not copies, (name, copies[:8])

