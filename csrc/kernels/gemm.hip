// MFMA GEMM for the Llama projections on gfx950 (MI355X / CDNA4).
//
//   C[M, N'] = epilogue( A[M, K] . W[N, K]^T )      fp16 in, fp32 accumulate
//
// A = activations (tokens x hidden, row-major), W = nn.Linear weight [out, in]
// (row-major, exactly as stored in the checkpoint) — both operands are
// K-contiguous, the natural MFMA layout.  The weights are consumed in the
// checkpoint's own row order: nothing is permuted on the host or by a relayout
// pass, so a layer streams from disk to HBM as plain DMA (runtime/stream.py).
//
// Kernels (one C ABI entry, fls_gemm, picks by shape):
//   * gemm_nt_v10 — 256 x 256 x 64 tile, 4 waves (one per SIMD), each wave
//     128 x 128 outputs in 256 AGPR accumulators (v_mfma_f32_16x16x32_f16: holds
//     a higher clock than 32x32x16 on random data, guide §5.4 r28).  Operands
//     staged global -> LDS by buffer_load_dwordx4 ... lds (LDS-DMA) with the XOR
//     chunk swizzle on the per-lane SOURCE address (guide T2 / rule 21), three
//     half-tile super-phases in flight, one counted vmcnt + raw s_barrier per
//     two phases, LDS fragment reads and DMA interleaved into the MFMA stream.
//     XCD-aware bijective block remap + grouped tile order (guide T1).
//   * gemm_nt_mid — 64 x 128 x 64 tiles, 3-deep LDS-DMA ring, for M too small
//     to fill 256 CUs with 256 x 256 tiles, and for odd K-tile counts (v10's
//     body is unrolled over two K-tiles); 4 waves, or 8 (two per SIMD) for
//     grids of about one block per CU, 64 or 128 rows; 64-column blocks.
//   * gemm_nt_generic — any shape (bounds-masked loads), for odd test shapes.
//
// The MFMA computes C^T tiles (A operand = W fragment, B operand = X fragment)
// so each lane holds 4 consecutive output columns of one row in each 16-column
// subtile (v10 pairs neighbouring subtiles into 16-byte stores with one
// v_permlane16_swap), and the epilogue partners live in the same lane:
//   RESID : C = acc (+ bias) + R          (R may alias C: in-place residual)
//   SWIGLU: W = [gate (I rows); up (I rows)] (HF gate_proj / up_proj stacked);
//           the W-tile loader reads logical rows interleaved per 16 (gate rows
//           16j.., up rows 16j..) so gate and up of one intermediate column sit
//           in neighbouring subtiles of the same lane; C has I = N/2 columns,
//           silu(gate) * up.
//   ROPE  : HF rotate-half on every head of the first rope_cols columns, in
//           natural head-dim order: the partner of column d of a head is
//           d + head_dim/2, which is 4 (hd 128) or 2 (hd 64) subtiles further
//           in the same lane; fp32 cos/sin tables [maxpos, hd/2], pos[m].
#include "gemm_v10.h"

namespace {

// ------------------------------------------------------------- generic
// Block = 4 waves; block tile 32 (M) x 256 (N); wave tile 32 x 64.
// Operands loaded straight from global with bounds masks (zero fill).
template <int EPI>
__global__ __launch_bounds__(256) void gemm_nt_generic(const half_t* __restrict__ A, const half_t* __restrict__ W,
                                                     half_t* __restrict__ C, int M, int N, int K, int lda, int ldw,
                                                     int ldc, Epi ep) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, grp = lane >> 4;
  const int m0 = blockIdx.x * 32;
  const bool rope128 = EPI == FLS_EPI_ROPE;
  // 128-column group of this wave and its position in it
  const int gbase = blockIdx.y * 256 + (wave >> 1) * 128;
  int ncol[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) ncol[t] = gbase + sub_col(rope128, wave & 1, t);
  floatx4 acc[2][4];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 32) {
    half8 wf[4], xf[2];
    const int kb = k0 + grp * 8;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int n = ncol[t] + fr;
      const int nr = EPI == FLS_EPI_SWIGLU ? gu_phys_row(n, ep.gu_rows) : n;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        wf[t][j] = (n < N && kb + j < K) ? W[(size_t)nr * ldw + kb + j] : (half_t)0.f;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int m = m0 + u * 16 + fr;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        xf[u][j] = (m < M && kb + j < K) ? A[(size_t)m * lda + kb + j] : (half_t)0.f;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[u][t] = mfma16x16x32(wf[t], xf[u], acc[u][t]);
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int m = m0 + u * 16 + fr;
    if (m >= M) continue;
    if constexpr (is_rope(EPI)) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (ncol[q + 2] + 16 <= N) store_rope_pair(C, ldc, m, ncol[q] + 4 * grp, acc[u][q], acc[u][q + 2], ep);
    } else {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int nf = ncol[2 * p];
        if (nf + 32 <= N) {
          store_pair_off<EPI>(C, ldc, m, nf, 4 * grp, acc[u][2 * p], acc[u][2 * p + 1], ep);
        } else if constexpr (EPI == FLS_EPI_NONE || EPI == FLS_EPI_RESID) {
          // ragged tail (N % 32 != 0): scalar stores
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int n = nf + h * 16 + 4 * grp + r;
              if (n < N) {
                float v = (h ? acc[u][2 * p + 1][r] : acc[u][2 * p][r]) * row_scale(ep, m);
                if (ep.bias) v += (float)ep.bias[n];
                if constexpr (EPI == FLS_EPI_RESID) v = v * ep.alpha + (float)ep.R[(size_t)m * ep.ldr + n];
                C[(size_t)m * ldc + n] = (half_t)v;
              }
            }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ mid-M
// For small / medium M (a few prompts, generation steps, LM heads with > 16
// scored rows) the 256x256 tiles leave most of the 256 CUs idle (7B QKV at
// M = 416: 96 blocks).  gemm_nt_mid uses 64 (M) x 128 (N) x 64 tiles: 4 waves
// in a 2 x 2 grid, each 32 x 64 outputs (2 x 4 MFMA 16x16x32 tiles, 32 fp32
// accumulators), operands staged by LDS-DMA (16 B per lane, XOR chunk swizzle
// on the source address) into a 3-deep ring with one counted vmcnt + raw
// barrier per K-tile; XCD-aware order puts every M tile of one N tile on the
// same XCD so each weight tile comes from HBM once and from L2 after that.
// Any K-tile count (the tail path for odd K / 64).
// One 16-column subtile of row m (columns c0 .. c0+3 of this lane): store_pair_off's arithmetic for
// one of its two subtiles, so 32-column mid blocks give the same bits (NONE / RESID epilogues)
template <int EPI>
__device__ __forceinline__ void store_one(half_t* __restrict__ C, int ldc, int m, int c0, const floatx4& acc,
                                          const Epi& ep) {
  static_assert(EPI == FLS_EPI_NONE || EPI == FLS_EPI_RESID, "pair epilogues need both subtiles");
  const float s = row_scale(ep, m);
  floatx4 a = acc * s;
  if (ep.bias) {
    const half4 ba = *(const half4*)(ep.bias + c0);
#pragma unroll
    for (int r = 0; r < 4; ++r) a[r] += (float)ba[r];
  }
  if constexpr (EPI == FLS_EPI_RESID) {
    const half4 ra = *(const half4*)(ep.R + (size_t)m * ep.ldr + c0);
#pragma unroll
    for (int r = 0; r < 4; ++r) a[r] = a[r] * ep.alpha + (float)ra[r];
  }
  half4 oa;
#pragma unroll
  for (int r = 0; r < 4; ++r) oa[r] = (half_t)a[r];
  *(half4*)(C + (size_t)m * ldc + c0) = oa;
}

// 8-wave 64-row mid blocks: column (in the 128-column block) of subtile t of wave column wn.  RoPE: the
// pair is a column and its partner hd/2 away (hd 128: 64 columns; hd 64: 32 in the same head).
__device__ __forceinline__ int mid8_col(int epi, int wn, int t) {
  if (epi == FLS_EPI_ROPE) return wn * 16 + t * 64;
  if (epi == EPI_ROPE64) return (wn >> 1) * 64 + (wn & 1) * 16 + t * 32;
  return wn * 32 + t * 16;
}

namespace mid {
constexpr int BMm = 64, BNm = 128, BKm = 64, NTm = 256, NSTAGE = 3;
// BNT: output columns per block, 128 (4 waves in 2 x 2, each 32 x 64) or 64 (each 32 x 32: twice the
// blocks for grids of less than one round of 128-column tiles); 32 with 8 waves (below)
// A rows 0 .. bmt-1 then W rows; LDS-DMA in 8-row (1 KiB) groups
constexpr int stage_bytes(int bnt, int bmt = BMm) { return (bmt + bnt) * BKm * 2; }
}  // namespace mid

// NST: LDS stages, NST - 1 K-tiles in flight ahead of the one being multiplied (3: 72 KB, two blocks
// per CU).  A 6-stage ring for one-round grids measured the same (70B generation-step shapes at
// M = 16-320, profiles/r6_decode/mid_ring): the blocks are not bound by their DMA latency.
// BNT = 64 blocks: a wave holds two 16-column subtiles (RoPE: a column and its partner hd/2 away; for
// head_dim 128 a block takes 32 columns of a head and their 32 partners).  Same fragments, MFMA and
// K order as BNT = 128, so the two are bitwise equal.
//
// WV = 8, two waves per SIMD.  With grids of about one block per CU (generation steps: the O / down /
// QKV projections at M = 16-320) a 4-wave block is bound by the latency chain of its single wave per
// SIMD (DMA wait, barrier, LDS reads, MFMAs); a second wave's MFMAs run under the first one's LDS
// reads (70B down at M = 160: 225 -> 196 us).  Shapes:
//   BMT = 64 : waves in 2 x 4, each 32 x 32 outputs (its two 16-column subtiles are a RoPE pair: a
//              column and its partner hd/2 away); 72 KB of LDS, two blocks per CU;
//   BMT = 128: waves in 4 x 2, each 32 x 64 as in the 4-wave block; 96 KB, one block per CU, half the
//              blocks (M = 320: 192 instead of 320, which left 64 CUs with two blocks);
//   BNT = 64 : waves in 4 x 2, each 16 x 32 (the 4-wave 64-column block's columns); M <= 64 layers
//              406 -> 377 us at M = 16, 431 -> 417 at M = 64 (profiles/r6_decode/mid8/bn64_*);
//   BNT = 32 : waves in 4 x 2, each 16 x 16 (plain / residual epilogues): 70B down at M = 64
//              155 -> 139 us (profiles/r6_decode/mid8/bn32_*).
// Same fragments, MFMA and K order in every shape, so all are bitwise equal.
template <int EPI, int NST, int BNT, int WV = 4, int BMT = mid::BMm>
__global__ __launch_bounds__(64 * WV) void gemm_nt_mid(const half_t* __restrict__ A, const half_t* __restrict__ W,
                                                     half_t* __restrict__ C, int M, int N, int K, int lda, int ldw,
                                                     int ldc, Epi ep) {
  using namespace mid;
  static_assert(WV == 4 || WV == 8, "4 or 8 waves");
  static_assert(BNT != 32 || (WV == 8 && (EPI == FLS_EPI_NONE || EPI == FLS_EPI_RESID)),
                "32-column blocks: 8 waves, one 16-column subtile per wave (no pair epilogues)");
  static_assert(BMT == 64 || (BMT == 128 && WV == 8 && BNT == 128), "128-row blocks: 8 waves, 128 columns");
  constexpr bool L24 = WV == 8 && BMT == 64 && BNT == 128;   // 2 x 4 waves of 32 x 32
  constexpr bool L42 = WV == 8 && BNT <= 64;                 // 4 x 2 waves of 16 x 32 (x 16 at BNT 32)
  constexpr int RW = L42 ? 16 : 32, U = RW / 16;             // rows per wave, 16-row subtiles per wave
  // 8-row LDS-DMA groups: waves 0 .. NG % WV - 1 take one more when they do not divide evenly
  constexpr int NG = (BMT + BNT) / 8, PER_WAVE = (NG + WV - 1) / WV, NG_REM = NG % WV;
  constexpr int STAGE = stage_bytes(BNT, BMT), NSUB = L24 ? 2 : BNT == 32 ? 1 : BNT / 32;
  extern __shared__ __attribute__((aligned(16))) char lds_mid[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, grp = lane >> 4;
  const int mt = (M + BMT - 1) / BMT, ntn = N / BNT;
  // XCD-aware bijective remap: logical tiles [xcd*q .. ) run on one XCD, M fastest
  int bid = blockIdx.x;
  {
    const int nwg = mt * ntn;
    const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    if (nwg >= 8) bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  }
  const int m0 = (bid % mt) * BMT;
  const int bn = bid / mt;
  const int n0 = bn * BNT;
  const int wm = L24 ? wave >> 2 : wave >> 1, wn = L24 ? wave & 3 : wave & 1;
  const int nk = K / BKm;
  const bool rope128 = EPI == FLS_EPI_ROPE;
  // BNT = 64 with RoPE over 128-wide heads: local W row l -> column of head bn / 2, quarter bn % 2
  const bool split_head = BNT == 64 && rope128;
  auto gcol = [&](int l) -> int {
    if (split_head) return (bn >> 1) * 128 + (bn & 1) * 32 + (l < 32 ? l : 64 + (l - 32));
    return n0 + l;
  };

  // this lane's LDS-DMA sources: group g = wave + WV*i covers tile rows 8*g .. 8*g+7
  const half_t* src[PER_WAVE];
  const int sub = lane >> 3;                       // row inside the 8-row group
  const int kc = ((lane & 7) ^ sub) * 8;           // source chunk pre-swizzled (read XORs it back)
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int g = min(wave + WV * i, NG - 1);       // (a group past NG is never issued)
    if (g < BMT / 8) {
      const int m = min(m0 + g * 8 + sub, M - 1);
      src[i] = A + (size_t)m * lda + kc;
    } else {
      const int n = gcol((g - BMT / 8) * 8 + sub);
      const int nr = EPI == FLS_EPI_SWIGLU ? gu_phys_row(n, ep.gu_rows) : n;
      src[i] = W + (size_t)nr * ldw + kc;
    }
  }
  // stage s takes K-tile kt (kt clamped to the last: a DMA past the end re-reads it into a stage
  // nobody reads again, so every wait is one constant count)
  auto stage = [&](int s, int kt) {
    char* base = lds_mid + (s % NST) * STAGE;
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i)
      if (NG_REM == 0 || i < PER_WAVE - 1 || wave < NG_REM)   // wave-uniform
        glds16(src[i] + (size_t)kt * BKm, base + (wave + WV * i) * 1024);
  };
  // local W rows of this wave's subtiles (RoPE: subtile t + NSUB / 2 is subtile t's partner)
  int wrow[NSUB];
#pragma unroll
  for (int t = 0; t < NSUB; ++t) {
    if constexpr (L24) wrow[t] = mid8_col(EPI, wn, t) + fr;
    else if constexpr (BNT == 128) wrow[t] = sub_col(rope128, wn, t) + fr;
    else if constexpr (BNT == 32) wrow[t] = wn * 16 + fr;
    else wrow[t] = (is_rope(EPI) ? wn * 16 + t * 32 : wn * 32 + t * 16) + fr;
  }

  floatx4 acc[U][NSUB];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int t = 0; t < NSUB; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int d = 0; d < NST - 1; ++d) stage(d, min(d, nk - 1));
  for (int kt = 0; kt < nk; ++kt) {
    // into the stage tile kt - 1 used (every wave passed that tile's closing barrier)
    stage(kt + NST - 1, min(kt + NST - 1, nk - 1));
    // tile kt landed
    if (NG_REM == 0 || wave < NG_REM) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 1) * PER_WAVE) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 1) * (PER_WAVE - 1)) : "memory");
    __builtin_amdgcn_s_barrier();                          // every wave's part of tile kt landed
    const char* Xs = lds_mid + (kt % NST) * STAGE;
    const char* Ws = Xs + BMT * BKm * 2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + grp;                          // logical 16-byte chunk of this lane
      half8 xf[U], wf[NSUB];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = wm * RW + u * 16 + fr;
        xf[u] = *(const half8*)(Xs + r * 128 + ((c ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int t = 0; t < NSUB; ++t) {
        const int r = wrow[t];
        wf[t] = *(const half8*)(Ws + r * 128 + ((c ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < NSUB; ++t) acc[u][t] = mfma16x16x32(wf[t], xf[u], acc[u][t]);
    }
    // WAR: the next iteration's DMA overwrites this stage; all reads are done
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");         // the redundant tail DMA, before LDS is handed on
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int m = m0 + wm * RW + u * 16 + fr;
    if (m >= M) continue;
    if constexpr (L24) {
      if constexpr (is_rope(EPI))
        store_rope_pair(C, ldc, m, n0 + mid8_col(EPI, wn, 0) + 4 * grp, acc[u][0], acc[u][1], ep);
      else
        store_pair_off<EPI>(C, ldc, m, n0 + wn * 32, 4 * grp, acc[u][0], acc[u][1], ep);
    } else if constexpr (BNT == 32) {
      store_one<EPI>(C, ldc, m, n0 + wn * 16 + 4 * grp, acc[u][0], ep);
    } else if constexpr (is_rope(EPI)) {
      if constexpr (BNT == 128) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
          store_rope_pair(C, ldc, m, n0 + sub_col(rope128, wn, q) + 4 * grp, acc[u][q], acc[u][q + 2], ep);
      } else {
        store_rope_pair(C, ldc, m, gcol(wn * 16) + 4 * grp, acc[u][0], acc[u][1], ep);
      }
    } else {
#pragma unroll
      for (int p = 0; p < NSUB / 2; ++p)
        store_pair_off<EPI>(C, ldc, m, n0 + wn * (BNT / 2) + p * 32, 4 * grp, acc[u][2 * p], acc[u][2 * p + 1], ep);
    }
  }
}

int g_order = 0;             // 0: by shape, else a fixed signed group size (fls_gemm_set_order)
int g_mid = 1;               // mid-M kernel on (fls_gemm_set_mid)
int g_mid_bn = 0;            // mid-M block columns: 0 auto, 64 / 128 forced where valid (fls_gemm_set_mid_bn)
int g_mid_waves = 0;         // 128-column mid blocks: 0 auto, 4 / 8 waves forced (fls_gemm_set_mid_waves)
int g_mid_rows = 0;          // 8-wave mid blocks' rows: 0 auto, 64 / 128 forced (fls_gemm_set_mid_rows)

template <int EPI, int NST, int BNT, int WV = 4, int BMT = mid::BMm>
void launch_mid(const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda, int ldw, int ldc,
                const Epi& ep, hipStream_t s) {
  static bool attr = false;
  constexpr int lds = NST * mid::stage_bytes(BNT, BMT);
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_nt_mid<EPI, NST, BNT, WV, BMT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  const int blocks = ((M + BMT - 1) / BMT) * (N / BNT);
  hipLaunchKernelGGL((gemm_nt_mid<EPI, NST, BNT, WV, BMT>), dim3(blocks), dim3(64 * WV), lds, s, A, W, C, M, N, K,
                     lda, ldw, ldc, ep);
}

template <int EPI>
void launch_main(int tiles, const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda, int ldw,
                 int ldc, const Epi& ep, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_nt_v10<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BUF);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_nt_v10<EPI>), dim3(tiles), dim3(256), 2 * BUF, s, A, W, C, M, N, K, lda, ldw, ldc, ep);
}


// ------------------------------------------------------------ split-K
// Small M (generation steps, small calls): a 256 x 256 tile grid of a few dozen tiles leaves most
// CUs idle and the mid-M kernel's 64-row tiles re-read every weight panel once per row tile.  Here
// each tile's K is cut into S slices (tiles x S >= one block per CU), every block streams its slice
// of the weight panel ONCE (the activation slice comes from L2) and writes fp32 partials
// (gemm_nt_v10<EPI_F32>); splitk_reduce_kernel sums the S slabs in a fixed order (deterministic)
// and applies the real epilogue (bias, residual, SwiGLU on the natural [gate; up] columns, RoPE
// with the partner column d + hd/2 of each head).
constexpr int SPLITK_MAX_M = 512;
int g_splitk = 1;            // split-K path for small M on (fls_gemm_set_splitk)
int ROW_CHUNK = 16384;       // main-path launches cover at most this many rows (fls_gemm_set_row_chunk)

template <int EPI>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int S, long long pstride,
                                                            int M, int N, half_t* __restrict__ C, int ldc, Epi ep) {
  const int units = N / 4;                                   // 4 raw columns per thread
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)M * units) return;
  const int m = (int)(idx / units), c = (int)(idx % units) * 4;
  const float rsc = row_scale(ep, m);
  auto sum4 = [&](int col) {
    floatx4 a = *(const floatx4*)(part + (size_t)m * N + col);
    for (int k = 1; k < S; ++k) a += *(const floatx4*)(part + (size_t)k * pstride + (size_t)m * N + col);
    return a * rsc;
  };
  auto bias4 = [&](floatx4& a, int col) {
    if (ep.bias) {
      const half4 b = *(const half4*)(ep.bias + col);
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] += (float)b[r];
    }
  };
  auto store4 = [&](const floatx4& a, int col) {
    half4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (half_t)a[r];
    *(half4*)(C + (size_t)m * ldc + col) = o;
  };
  if constexpr (EPI == FLS_EPI_SWIGLU) {
    const int I = N / 2;
    if (c >= I) return;                                      // gate threads do both halves
    const floatx4 g = sum4(c), u = sum4(I + c);
    floatx4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = silu(g[r]) * u[r];
    store4(o, c);
  } else if constexpr (is_rope(EPI)) {
    const int hd = ep.head_dim, half_hd = hd >> 1, d = c % hd;
    if (c < ep.rope_cols && d >= half_hd) return;            // the partner thread rotates this pair
    floatx4 a = sum4(c);
    bias4(a, c);
    if (c >= ep.rope_cols) {
      store4(a, c);
      return;
    }
    floatx4 b = sum4(c + half_hd);
    bias4(b, c + half_hd);
    const int p = ep.pos[m];
    const floatx4 cs = *(const floatx4*)(ep.cos_t + (size_t)p * half_hd + d);
    const floatx4 sn = *(const floatx4*)(ep.sin_t + (size_t)p * half_hd + d);
    floatx4 y1, y2;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      y1[r] = a[r] * cs[r] - b[r] * sn[r];
      y2[r] = b[r] * cs[r] + a[r] * sn[r];
    }
    store4(y1, c);
    store4(y2, c + half_hd);
  } else {
    floatx4 a = sum4(c);
    bias4(a, c);
    if constexpr (EPI == FLS_EPI_RESID) {
      const half4 rr = *(const half4*)(ep.R + (size_t)m * ep.ldr + c);
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = a[r] * ep.alpha + (float)rr[r];
    }
    store4(a, c);
  }
}

#include "gemm_skinny.h"

// ss[m * ss_ld + j] = sum over columns [128 j, 128 j + 128) of C[m, :]^2 (fp32 of the fp16 values):
// the per-row partials of the v10 / v11 residual epilogue (Epi::ss) for the GEMM paths whose own
// epilogue does not write them (skinny, split-K, mid-M, generic: small M), and the fused norm's
// statistic of a hidden state without partials (fls_row_ss).  One wave per (16 rows, 128 columns) in
// the epilogue's lane layout -- lane (row fr, group g) holds columns 32 p + 4 g + r and 32 p + 16 +
// 4 g + r, p, r < 4 -- through the same ss_accum_pair and row_sum_4groups: bitwise the epilogue's.
__global__ __launch_bounds__(256) void ss_partials_kernel(const half_t* __restrict__ C, int ldc, int M, int nparts,
                                                          float* __restrict__ ss, int ss_ld) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int rgroups = (M + 15) / 16;
  if (w >= rgroups * nparts) return;                // wave-uniform
  const int fr = lane & 15, grp = lane >> 4;
  const int m = (w / nparts) * 16 + fr, j = w % nparts;
  const half_t* p0 = C + (size_t)min(m, M - 1) * ldc + j * 128 + grp * 4;
  float sq = 0.f;
#pragma unroll
  for (int p = 0; p < 4; ++p) sq = ss_accum_pair(sq, *(const half4*)(p0 + p * 32), *(const half4*)(p0 + p * 32 + 16));
  sq = row_sum_4groups(sq);                         // every lane (permlane swaps)
  if (grp == 0 && m < M) ss[(size_t)m * ss_ld + j] = sq;
}

// the fused norm's statistic straight from x, one wave per row: lane j computes the 128-column
// partials j, j + 64, ... itself, with ss_partials_kernel's per-lane FMA chains (one per 4-column group
// g) combined as row_sum_4groups does, (g0 + g2) + (g1 + g3), and sums them in rstd_from_ss_kernel's
// order (lane j takes parts j, j + 64, ..., then warp_sum): the same bits as fls_row_ss followed by
// fls_rstd_from_ss, in one launch (generation steps run two per layer).  The 16-row lane layout of
// the GEMM epilogue, kept here first, cost 16 us per launch at any row count (16 rows per block, 32
// rows' worth of scattered 32-byte pieces per load); lane-per-part loads stream each row.
constexpr int ROW_STAT_MAX_PARTS = 128;              // H <= 16,384
__global__ __launch_bounds__(256) void row_stat_kernel(const half_t* __restrict__ x, int ldx, int M, int nparts, int H,
                                                       float eps, float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;                               // wave-uniform (no block barrier)
  const half_t* row = x + (size_t)m * ldx;
  float v = 0.f;
  for (int j = lane; j < nparts; j += 64) {
    half4 q[32];                                    // the part's 128 columns
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const half8 c = *(const half8*)(row + j * 128 + k * 8);
      q[2 * k] = c.lo;
      q[2 * k + 1] = c.hi;
    }
    float sg[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float sq = 0.f;
#pragma unroll
      for (int p = 0; p < 4; ++p) sq = ss_accum_pair(sq, q[p * 8 + g], q[p * 8 + 4 + g]);
      sg[g] = sq;
    }
    v += (sg[0] + sg[2]) + (sg[1] + sg[3]);
  }
  v = warp_sum(v);
  if (lane == 0) rstd[m] = rsqrtf(v / (float)H + eps);
}

void ss_partials_raw(const half_t* C, int ldc, int M, int N, float* ss, int ss_ld, hipStream_t s) {
  if (!ss || M <= 0) return;
  const int waves = ((M + 15) / 16) * (N / 128);
  hipLaunchKernelGGL(ss_partials_kernel, dim3((waves + 3) / 4), dim3(256), 0, s, C, ldc, M, N / 128, ss, ss_ld);
}

void ss_partials(const half_t* C, int ldc, int M, int N, const Epi& ep, hipStream_t s) {
  ss_partials_raw(C, ldc, M, N, ep.ss, ep.ss_ld, s);
}

// -> slices per tile (0: split-K not applicable / no room in the workspace)
int splitk_slices(int M, int N, int K, size_t tiles, size_t ws_bytes) {
  if (tiles >= 128) return 0;
  const int nk = K / BK;
  int best = 0;
  for (int S = 2; S <= 32; S *= 2) {
    if (nk % (2 * S) || (size_t)S * M * N * 4 > ws_bytes) break;
    best = S;
    if (tiles * S >= 256) break;                           // one block per CU reached
  }
  return best;
}

template <int EPI>
int launch(const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda, int ldw, int ldc,
           const Epi& ep, hipStream_t s, void* ws, size_t ws_bytes) {
  const bool mid_ok = N % mid::BNm == 0 && K % mid::BKm == 0 && lda % 8 == 0 && ldw % 8 == 0;
  const size_t tiles256 = (size_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  // 32-bit per-lane DMA offsets (X rows; SWIGLU up-block rows)
  const bool offs32 = (size_t)M * lda * 2 < (1ull << 32) &&
                      (EPI != FLS_EPI_SWIGLU || (size_t)(N / 2 + BN) * ldw * 2 < (1ull << 32));
  // the v10 epilogues store (and load the residual) 16 B per lane
  const bool wide_ok = ldc % 8 == 0 && ((uintptr_t)C & 15) == 0 &&
                       (EPI != FLS_EPI_RESID || (ep.ldr % 8 == 0 && ((uintptr_t)ep.R & 15) == 0));
  const bool main_ok = N % BN == 0 && K % BK == 0 && (K / BK) % 2 == 0 && lda % 8 == 0 && ldw % 8 == 0 && offs32 &&
                       wide_ok;
  // Too few 256x256 tiles for 256 CUs -> 64x128 tiles.  Measured crossover (profiles/r1_gemm_mid):
  // the mid kernel wins below ~128 main tiles, and at M <= 64 (3/4 of every 256-row tile wasted)
  // up to 512; above that its lower L2 reuse (43 vs 128 FLOP per staged byte) costs more than the
  // idle CUs.  It is also the path for odd K-tile counts.
  // split-K for small M: the whole weight read once, every CU streaming (see splitk_reduce_kernel)
  const bool split_ok = g_splitk && ws && M <= SPLITK_MAX_M && N % BN == 0 && K % BK == 0 && lda % 8 == 0 &&
                        ldw % 8 == 0 && (size_t)M * lda * 2 < (1ull << 32) && ldc % 4 == 0 &&
                        ((uintptr_t)C & 7) == 0 && ((uintptr_t)ws & 15) == 0 &&
                        (EPI != FLS_EPI_RESID || (ep.ldr % 4 == 0 && ((uintptr_t)ep.R & 7) == 0));
  if (!ep.row_exact) {
    const int rc = try_skinny<EPI>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, ws, ws_bytes);
    if (rc > 0) ss_partials(C, ldc, M, N, ep, s);
    if (rc) return rc > 0 ? 0 : rc;
  }
  const int S = split_ok && !ep.row_exact ? splitk_slices(M, N, K, tiles256, ws_bytes) : 0;
  if (S >= 2 && (M > 64 || tiles256 * S >= 128)) {
    static bool attr_f32 = false;
    if (!attr_f32) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_v10<EPI_F32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * BUF);
      attr_f32 = true;
    }
    Epi e = ep;
    const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN;
    e.order = g_order ? g_order : auto_order(tiles_m, tiles_n);
    e.ksplit = S;
    e.kslice = K / S;
    e.part_stride = (long long)M * N;
    float* part = (float*)ws;
    hipLaunchKernelGGL((gemm_nt_v10<EPI_F32>), dim3((int)tiles256 * S), dim3(256), 2 * BUF, s, A, W, (half_t*)part, M,
                       N, K / S, lda, ldw, N, e);
    FLS_CHECK_LAUNCH();
    const long long threads = (long long)M * (N / 4);
    hipLaunchKernelGGL(splitk_reduce_kernel<EPI>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, part, S,
                       e.part_stride, M, N, C, ldc, e);
    FLS_CHECK_LAUNCH();
    ss_partials(C, ldc, M, N, ep, s);
    FLS_CHECK_LAUNCH();
    return 0;
  }
  if (mid_ok && (!main_ok || (g_mid && (tiles256 < 128 || (M <= 64 && tiles256 < 512))))) {
    // 64-column blocks for a single row tile whose 128-column grid fills less than one round of the
    // 256 CUs: 70B generation steps with 8 prompts (M = 40) 39.7 vs 46.7 ms per step; with 32 prompts
    // (M = 160, three row tiles) the 128-column blocks are faster, 53 vs 55.5 ms (profiles/r6_decode/
    // mid_bn: in-graph steps, cold weights; a same-weights GEMM loop favoured 64 there too)
    const int blocks128 = ((M + mid::BMm - 1) / mid::BMm) * (N / mid::BNm);
    const bool bn64_ok = N % 64 == 0 && (EPI != FLS_EPI_ROPE || N % 128 == 0);
    // (and, since the 8-wave blocks, for two row tiles of at most ~1.25 rounds: 70B at M = 96, down
    // 193 -> 147 us, O 49 -> 36 us; profiles/r6_decode/mid8/bn64_m96_gemm_bench.log)
    const int blocks64_ = ((M + mid::BMm - 1) / mid::BMm) * (N / 64);
    const bool bn64 = bn64_ok && (g_mid_bn == 64 || (g_mid_bn == 0 && ((blocks128 < 256 && M <= mid::BMm) ||
                                                                       (M <= 2 * mid::BMm && blocks64_ <= 320))));
    // 8 waves for grids of < 2 rounds of 64-row blocks; 128-row blocks when 64-row ones take more than
    // one round, 128-row ones fit in one and K is long (profiles/r6_decode/mid8, 70B at M = 320: down
    // 343 -> 276 us; the K = 8,192 projections ran 5-10% slower with 128 rows)
    const bool w8 = g_mid_waves == 8 || (g_mid_waves == 0 && blocks128 < 512);
    const int rows128 = (M + 127) / 128 * (N / mid::BNm);
    const bool r128 = g_mid_rows == 128 || (g_mid_rows == 0 && blocks128 > 256 && rows128 <= 256 && K >= 16384);
    const int blocks64 = ((M + mid::BMm - 1) / mid::BMm) * (N / 64);
    const bool w8_64 = g_mid_waves == 8 || (g_mid_waves == 0 && blocks64 < 512);
    // 32-column blocks (NONE / RESID epilogues) when even 64-column ones leave CUs idle: the 70B O and
    // down projections of generation steps with <= 12 prompts (M <= 64: 128 -> 256 blocks)
    constexpr bool bn32_epi = EPI == FLS_EPI_NONE || EPI == FLS_EPI_RESID;
    const bool bn32 = bn32_epi && N % 32 == 0 && g_mid_waves != 4 &&
                      (g_mid_bn == 32 || (g_mid_bn == 0 && M <= mid::BMm && blocks64 < 256));
    if constexpr (bn32_epi) {
      if (bn32) {
        launch_mid<EPI, mid::NSTAGE, 32, 8>(A, W, C, M, N, K, lda, ldw, ldc, ep, s);
        FLS_CHECK_LAUNCH();
        ss_partials(C, ldc, M, N, ep, s);
        FLS_CHECK_LAUNCH();
        return 0;
      }
    }
    if (bn64 && w8_64)
      launch_mid<EPI, mid::NSTAGE, 64, 8>(A, W, C, M, N, K, lda, ldw, ldc, ep, s);
    else if (bn64)
      launch_mid<EPI, mid::NSTAGE, 64>(A, W, C, M, N, K, lda, ldw, ldc, ep, s);
    else if (w8 && r128)
      launch_mid<EPI, mid::NSTAGE, 128, 8, 128>(A, W, C, M, N, K, lda, ldw, ldc, ep, s);
    else if (w8)
      launch_mid<EPI, mid::NSTAGE, 128, 8>(A, W, C, M, N, K, lda, ldw, ldc, ep, s);
    else
      launch_mid<EPI, mid::NSTAGE, 128>(A, W, C, M, N, K, lda, ldw, ldc, ep, s);
    FLS_CHECK_LAUNCH();
    ss_partials(C, ldc, M, N, ep, s);
    FLS_CHECK_LAUNCH();
    return 0;
  }
  if (!main_ok) {
    dim3 grid((M + 31) / 32, (N + 255) / 256);
    hipLaunchKernelGGL(gemm_nt_generic<EPI>, grid, dim3(256), 0, s, A, W, C, M, N, K, lda, ldw, ldc, ep);
    FLS_CHECK_LAUNCH();
    ss_partials(C, ldc, M, N, ep, s);
    FLS_CHECK_LAUNCH();
    return 0;
  }
  // Row chunks of <= ROW_CHUNK rows: with more rows the activation panel (M x K) outgrows the 256 MB
  // Infinity Cache and the N-grouped tile order re-reads it from HBM once per group of weight
  // columns.  70B O projection over 43,008 rows: one launch 1,361 TFLOP/s, three of 14,336 rows
  // 1,421 (gate/up + SwiGLU 1,325 -> 1,430; profiles/r3_gemm, scripts/gemm_m_chunks.py).
  // Only when every chunk still fills the chip (>= 256 tiles), so each piece stays on this path.
  const int n_chunks = (M + ROW_CHUNK - 1) / ROW_CHUNK;
  const int step = ((M + n_chunks - 1) / n_chunks + BM - 1) / BM * BM;
  if (M > ROW_CHUNK && (size_t)(step / BM) * (N / BN) >= 256) {
    for (int r0 = 0; r0 < M; r0 += step) {
      Epi e = ep;
      if (e.pos) e.pos += r0;
      if (e.R) e.R += (size_t)r0 * e.ldr;
      if (e.ss) e.ss += (size_t)r0 * e.ss_ld;
      if (e.rs) e.rs += r0;                  // (the fused norm's per-row statistic follows its rows)
      const int rc = launch<EPI>(A + (size_t)r0 * lda, W, C + (size_t)r0 * ldc, min(step, M - r0), N, K, lda, ldw,
                                 ldc, e, s, ws, ws_bytes);
      if (rc) return rc;
    }
    return 0;
  }
  // One block per tile, dispatched by the hardware as CUs free up.  A persistent form (one block
  // per CU walking its tiles, the next tile's prologue DMA under this tile's epilogue) measured
  // 1.1-3.9% slower on every 70B / 7B shape once the tile order was XCD-aware (profiles/r2_gemm).
  const int tiles = (int)tiles256;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN;
  int order = g_order;
  if (order == 0) order = auto_order(tiles_m, tiles_n);
  Epi e = ep;
  e.order = order;
  launch_main<EPI>(tiles, A, W, C, M, N, K, lda, ldw, ldc, e, s);
  FLS_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int fls_kernels_version(void) { return 33; }

// tile order: 0 = by shape (default); g > 0: groups of g M tiles; g < 0: groups of -g N tiles (A/B, tests)
extern "C" int fls_gemm_set_order(int order) {
  const int old = g_order;
  g_order = order;
  return old;
}

// skinny-M path (gemm_skinny.h): 0 off, 1 auto (default), 2 every M <= 256 it supports; blocks: the
// K-split block target (0: the whole-round rule, the default); returns the previous mode
extern "C" int fls_gemm_set_skinny(int mode, int blocks) {
  const int old = g_skinny;
  g_skinny = mode < 0 ? 0 : mode > 2 ? 2 : mode;
  g_skinny_blocks = blocks > 0 ? blocks : 0;
  return old;
}

// skinny-M weight rows per block: 0 auto (default), 128 or 256 where supported; returns the previous
extern "C" int fls_gemm_set_skinny_bn(int bn) {
  const int old = g_skinny_bn;
  g_skinny_bn = bn == 128 || bn == 256 ? bn : 0;
  return old;
}

// split-K path for small M on (1, default) or off (0; tests / A-B)
extern "C" int fls_gemm_set_splitk(int on) {
  const int old = g_splitk;
  g_splitk = on ? 1 : 0;
  return old;
}

// rows per main-path launch (0: unlimited; default 16384)
extern "C" int fls_gemm_set_row_chunk(int rows) {
  const int old = ROW_CHUNK;
  ROW_CHUNK = rows > 0 ? rows : (1 << 30);
  return old;
}

// per-row partial sums of squares of an fp16 [rows, H] matrix, one fp32 per 128 columns (H % 128 == 0):
// the residual GEMM epilogue's partials, bitwise, for a hidden state that arrived without them
extern "C" int fls_row_ss(const void* x, int ldx, int rows, int H, float* ss, int ss_ld, fls_stream_t s) {
  if (rows <= 0) return 0;
  if (H % 128 || ldx % 4 || ((uintptr_t)x & 7) || ss_ld < H / 128) return -2;
  ss_partials_raw((const half_t*)x, ldx, rows, H, ss, ss_ld, (hipStream_t)s);
  FLS_CHECK_LAUNCH();
  return 0;
}

// rstd[r] = rsqrt(mean(x[r]^2) + eps) for an fp16 [rows, H] matrix (H % 128 == 0, H <= 16,384), bitwise
// fls_row_ss + fls_rstd_from_ss (the fused norm's statistic without a residual GEMM's partials)
extern "C" int fls_row_stat(const void* x, int ldx, int rows, int H, float eps, float* rstd, fls_stream_t s) {
  if (rows <= 0) return 0;
  if (H % 128 || H / 128 > ROW_STAT_MAX_PARTS || ldx % 8 || ((uintptr_t)x & 15)) return -2;
  hipLaunchKernelGGL(row_stat_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)s, (const half_t*)x, ldx, rows,
                     H / 128, H, eps, rstd);
  FLS_CHECK_LAUNCH();
  return 0;
}

// mid-M block columns: 0 auto (default), 32, 64 or 128 forced where valid (tests / A-B; 32: NONE / RESID
// epilogues, 8 waves); returns the previous
extern "C" int fls_gemm_set_mid_bn(int bn) {
  const int old = g_mid_bn;
  g_mid_bn = bn == 32 || bn == 64 || bn == 128 ? bn : 0;
  return old;
}

// 128-column mid-M blocks: 0 auto (default: 8 waves for grids of < 512 blocks), 4 or 8 waves forced
// (tests / A-B); returns the previous
extern "C" int fls_gemm_set_mid_waves(int waves) {
  const int old = g_mid_waves;
  g_mid_waves = waves == 4 || waves == 8 ? waves : 0;
  return old;
}

// 8-wave mid-M blocks' rows: 0 auto (default: 128 when 64-row blocks would take more than one round
// and 128-row ones fit in one), 64 or 128 forced (tests / A-B); returns the previous
extern "C" int fls_gemm_set_mid_rows(int rows) {
  const int old = g_mid_rows;
  g_mid_rows = rows == 64 || rows == 128 ? rows : 0;
  return old;
}

// mid-M kernel for small grids on (1, default) or off (0; tests)
extern "C" int fls_gemm_set_mid(int on) {
  const int old = g_mid;
  g_mid = on ? 1 : 0;
  return old;
}

// gemm_v11.hip: the 384 x 256 tile for large projections (returns 1 when it took the GEMM)
extern "C" int fls_gemm_v11_try(const void* A, const void* W, void* C, const void* R, int M, int N, int K, int lda,
                                int ldw, int ldc, int ldr, int epi, const int* pos, const float* cos_t,
                                const float* sin_t, int rope_cols, int head_dim, const void* bias,
                                const float* rscale, float alpha, float* ss, int ss_ld, fls_stream_t s);

extern "C" int fls_gemm(const void* A, const void* W, void* C, const void* R, int M, int N, int K, int lda, int ldw,
                        int ldc, int ldr, int epi, const int* pos, const float* cos_t, const float* sin_t,
                        int rope_cols, int head_dim, const void* bias, const float* rscale, float alpha, float* ss,
                        int ss_ld, void* ws, uint64_t ws_bytes, fls_stream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const int row_exact = (epi & FLS_GEMM_ROW_EXACT) ? 1 : 0;
  epi &= 0xff;
  // row partial sums of squares: residual GEMMs only, one per 128 output columns
  if (ss && (epi != FLS_EPI_RESID || N % 128 || ss_ld < N / 128)) return -7;
  if (bias && epi == FLS_EPI_SWIGLU) return -4;
  if ((epi == FLS_EPI_SWIGLU || epi == FLS_EPI_ROPE) && (N % 32)) return -2;
  if (epi == FLS_EPI_ROPE && ((head_dim != 64 && head_dim != 128) || rope_cols % head_dim || N % head_dim))
    return -3;
  {
    const int rc = fls_gemm_v11_try(A, W, C, R, M, N, K, lda, ldw, ldc, ldr, epi, pos, cos_t, sin_t, rope_cols,
                                    head_dim, bias, rscale, alpha, ss, ss_ld, s);
    if (rc) return rc > 0 ? 0 : rc;
  }
  Epi ep{(const half_t*)R, ldr, pos, cos_t, sin_t, rope_cols, head_dim, (const half_t*)bias, N / 2, 0,
         nullptr, nullptr, nullptr, 0, 0};
  ep.rs = rscale;
  ep.alpha = alpha;
  ep.ss = ss;
  ep.ss_ld = ss_ld;
  ep.row_exact = row_exact;
  auto a = (const half_t*)A;
  auto w = (const half_t*)W;
  auto c = (half_t*)C;
  auto st = (hipStream_t)s;
  switch (epi) {
    case FLS_EPI_NONE: return launch<FLS_EPI_NONE>(a, w, c, M, N, K, lda, ldw, ldc, ep, st, ws, ws_bytes);
    case FLS_EPI_RESID: return launch<FLS_EPI_RESID>(a, w, c, M, N, K, lda, ldw, ldc, ep, st, ws, ws_bytes);
    case FLS_EPI_SWIGLU: return launch<FLS_EPI_SWIGLU>(a, w, c, M, N, K, lda, ldw, ldc, ep, st, ws, ws_bytes);
    case FLS_EPI_ROPE:
      return head_dim == 128 ? launch<FLS_EPI_ROPE>(a, w, c, M, N, K, lda, ldw, ldc, ep, st, ws, ws_bytes)
                             : launch<EPI_ROPE64>(a, w, c, M, N, K, lda, ldw, ldc, ep, st, ws, ws_bytes);
  }
  return -1;
}
