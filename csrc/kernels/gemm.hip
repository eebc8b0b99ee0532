// MFMA GEMM for the Llama projections on gfx950 (MI355X / CDNA4).
//
//   C[M, N'] = epilogue( A[M, K] . W[N, K]^T )      fp16 in, fp32 accumulate
//
// A = activations (tokens x hidden, row-major), W = nn.Linear weight [out, in]
// (row-major) — both operands are K-contiguous, the natural MFMA layout.
//
// Main kernel (M any, N % 256 == 0, K % 64 == 0):
//   * 256 x 256 x 64 block tile, 512 threads = 8 waves (4 along N x 2 along M),
//     each wave 64 (N) x 128 (M) = 4 x 8 tiles of v_mfma_f32_16x16x32_f16
//     (16x16x32 holds a higher clock than 32x32x16 on random data — guide §5.4 r28);
//   * operands staged global -> LDS by global_load_lds_dwordx4 (LDS-DMA, no
//     VGPR round trip), double-buffered (2 x 64 KiB), with the XOR chunk
//     swizzle applied on the per-lane SOURCE address so ds_read_b128 fragment
//     reads are bank-conflict free (guide T2 / rule 21);
//   * the MFMA computes C^T tiles (A operand = W fragment, B operand = X
//     fragment) so each lane ends up with 4 consecutive output columns of one
//     row: 8-byte stores, and the epilogue partners (RoPE pair, gate/up) sit
//     in neighbouring 16-column subtiles of the SAME lane — fused in registers;
//   * XCD-aware bijective block remap + grouped (8 M-tiles) ordering so the
//     32 blocks resident on one XCD share W/X K-panels in that XCD's L2.
// Epilogues: NONE, RESID (C = acc + R, R may alias C), SWIGLU (gate/up rows
// interleaved per 16 -> C has N/2 columns), ROPE (rotate RoPE-pair-permuted
// q/k columns < rope_cols with fp32 cos/sin tables).
//
// Generic fallback kernel (any M, N % 16 == 0, K) for odd test shapes.
#include "common.h"
#include "fls.h"

#include <cstdlib>

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int TILE_BYTES = BM * BK * 2;          // 32 KiB per operand tile
constexpr int STAGE_BYTES = 2 * TILE_BYTES;       // W + X
constexpr int LDS_BYTES = 2 * STAGE_BYTES;        // double buffered: 128 KiB

struct Epi {
  const half_t* R;
  int ldr;
  const int* pos;
  const float* cos_t;
  const float* sin_t;
  int rope_cols;
  int head_dim;
};

// Store one pair of 16-column subtiles (cols n_first + 4*grp + r and +16)
// for output row m.  acc_a: first subtile, acc_b: second (its partner).
template <int EPI>
__device__ __forceinline__ void store_pair(half_t* __restrict__ C, int ldc, int m, int n_first, int grp,
                                           const floatx4& acc_a, const floatx4& acc_b, const Epi& ep) {
  const int c0 = n_first + 4 * grp;
  if constexpr (EPI == FLS_EPI_SWIGLU) {
    // pair = (gate, up) of intermediate columns [n_first/2, n_first/2 + 16)
    const int oc = n_first / 2 + 4 * grp;
    half4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (half_t)(silu(acc_a[r]) * acc_b[r]);
    *(half4*)(C + (size_t)m * ldc + oc) = o;
    return;
  } else {
    floatx4 a = acc_a, b = acc_b;
    if constexpr (EPI == FLS_EPI_ROPE) {
      if (n_first < ep.rope_cols) {
        const int hd = ep.head_dim, half_hd = hd >> 1;
        const int o = c0 % hd;
        const int f0 = (o >> 5) * 16 + (o & 15);
        const int p = ep.pos[m];
        const float* cr = ep.cos_t + (size_t)p * half_hd + f0;
        const float* sr = ep.sin_t + (size_t)p * half_hd + f0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float cs = cr[r], sn = sr[r];
          const float x1 = acc_a[r], x2 = acc_b[r];
          a[r] = x1 * cs - x2 * sn;
          b[r] = x2 * cs + x1 * sn;
        }
      }
    }
    if constexpr (EPI == FLS_EPI_RESID) {
      const half4 ra = *(const half4*)(ep.R + (size_t)m * ep.ldr + c0);
      const half4 rb = *(const half4*)(ep.R + (size_t)m * ep.ldr + c0 + 16);
#pragma unroll
      for (int r = 0; r < 4; ++r) { a[r] += (float)ra[r]; b[r] += (float)rb[r]; }
    }
    half4 oa, ob;
#pragma unroll
    for (int r = 0; r < 4; ++r) { oa[r] = (half_t)a[r]; ob[r] = (half_t)b[r]; }
    *(half4*)(C + (size_t)m * ldc + c0) = oa;
    *(half4*)(C + (size_t)m * ldc + c0 + 16) = ob;
  }
}

// ABL (ablation, microbenchmarks only): bit0 = no LDS-DMA in the K loop,
// bit1 = no fragment ds_reads (stale registers), bit2 = no MFMAs.
template <int EPI, int ABL = 0, int ORD = 0>
__global__ __launch_bounds__(NT, 2) void gemm_nt_256x256(const half_t* __restrict__ A, const half_t* __restrict__ W,
                                                        half_t* __restrict__ C, int M, int N, int K, int lda, int ldw,
                                                        int ldc, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // ---- XCD-aware bijective remap, then grouped tile order
  const int nwg = gridDim.x;
  int bid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  }
  const int tiles_m = (M + BM - 1) / BM;
  const int tiles_n = N / BN;
  int tm, tn;
  if constexpr (ORD == 0) {          // groups of 8 M-tiles sweep N (W streamed per group)
    constexpr int GROUP_M = 8;
    const int group = bid / (GROUP_M * tiles_n);
    const int first_m = group * GROUP_M;
    const int gsz = min(tiles_m - first_m, GROUP_M);
    const int in_g = bid - group * GROUP_M * tiles_n;
    tm = first_m + in_g % gsz;
    tn = in_g / gsz;
  } else {                           // groups of 8 N-tiles sweep M (X streamed per group)
    constexpr int GROUP_N = 8;
    const int group = bid / (GROUP_N * tiles_m);
    const int first_n = group * GROUP_N;
    const int gsz = min(tiles_n - first_n, GROUP_N);
    const int in_g = bid - group * GROUP_N * tiles_m;
    tn = first_n + in_g % gsz;
    tm = in_g / gsz;
  }
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- staging sources: each wave fills 4 x 1 KiB of the W tile and of the X tile.
  const int lr = lane >> 3;              // row inside the 8-row piece
  const int lc = (lane & 7) ^ lr;        // source chunk (inverse swizzle on the source)
  const half_t* wsrc[4];
  const half_t* xsrc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int piece = wave * 4 + j;
    const int rw = n0 + piece * 8 + lr;
    const int rx = min(m0 + piece * 8 + lr, M - 1);
    wsrc[j] = W + (size_t)rw * ldw + lc * 8;
    xsrc[j] = A + (size_t)rx * lda + lc * 8;
  }
  auto stage = [&](int buf, int k0) {
    char* base = smem + buf * STAGE_BYTES;
#pragma unroll
    for (int j = 0; j < 4; ++j) glds16(wsrc[j] + k0, base + (wave * 4 + j) * 1024);
#pragma unroll
    for (int j = 0; j < 4; ++j) glds16(xsrc[j] + k0, base + TILE_BYTES + (wave * 4 + j) * 1024);
  };

  const int wn = wave & 3, wm = wave >> 2;
  const int fr = lane & 15, grp = lane >> 4;
  floatx4 acc[8][4];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};

  // fragment byte offsets inside a stage (row*128 + swizzled chunk*16)
  const int wrow0 = wn * 64 + fr;
  const int xrow0 = wm * 128 + fr;
  const int swz = lane & 7;  // row & 7 == fr & 7 for every fragment row

  const int nk = K / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  half8 wf[4], xf[8];
#pragma unroll
  for (int t = 0; t < 4; ++t) wf[t] = half8{};
#pragma unroll
  for (int u = 0; u < 8; ++u) xf[u] = half8{};
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (!(ABL & 1) && kt + 1 < nk) stage(cur ^ 1, (kt + 1) * BK);
    const char* Ws = smem + cur * STAGE_BYTES;
    const char* Xs = Ws + TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = ((s * 4 + grp) ^ swz) << 4;
      if (!(ABL & 2)) {
#pragma unroll
        for (int t = 0; t < 4; ++t) wf[t] = *(const half8*)(Ws + (wrow0 + t * 16) * 128 + ch);
#pragma unroll
        for (int u = 0; u < 8; ++u) xf[u] = *(const half8*)(Xs + (xrow0 + u * 16) * 128 + ch);
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) asm volatile("" : "+v"(wf[t]));
#pragma unroll
        for (int u = 0; u < 8; ++u) asm volatile("" : "+v"(xf[u]));
      }
      if (!(ABL & 4)) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[u][t] = mfma16x16x32(wf[t], xf[u], acc[u][t]);
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) asm volatile("" :: "v"(wf[t]));
#pragma unroll
        for (int u = 0; u < 8; ++u) asm volatile("" :: "v"(xf[u]));
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: lane holds C[m][n_sub + 4*grp + r]
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int m = m0 + wm * 128 + u * 16 + fr;
    if (m < M) {
#pragma unroll
      for (int p = 0; p < 2; ++p)
        store_pair<EPI>(C, ldc, m, n0 + wn * 64 + p * 32, grp, acc[u][2 * p], acc[u][2 * p + 1], ep);
    }
  }
}

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
  const int nw = blockIdx.y * 256 + wave * 64;
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
      const int n = nw + t * 16 + fr;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        wf[t][j] = (n < N && kb + j < K) ? W[(size_t)n * ldw + kb + j] : (half_t)0.f;
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
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int nf = nw + p * 32;
      if (nf + 32 <= N) {
        store_pair<EPI>(C, ldc, m, nf, grp, acc[u][2 * p], acc[u][2 * p + 1], ep);
      } else if constexpr (EPI == FLS_EPI_NONE || EPI == FLS_EPI_RESID) {
        // ragged tail (N % 32 != 0): scalar stores
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int n = nf + h * 16 + 4 * grp + r;
            if (n < N) {
              float v = h ? acc[u][2 * p + 1][r] : acc[u][2 * p][r];
              if constexpr (EPI == FLS_EPI_RESID) v += (float)ep.R[(size_t)m * ep.ldr + n];
              C[(size_t)m * ldc + n] = (half_t)v;
            }
          }
      }
    }
  }
}

// ------------------------------------------------------------------ v3
// Ping-pong: the 8 waves form two groups (waves 0-3 / 4-7; the hardware puts
// one wave of each group on every SIMD).  Group 1 runs one barrier-slot
// behind group 0, so in every slot one wave per SIMD issues the 64 MFMAs of
// a whole 256x256x64 K-tile (1024 matrix-pipe cycles) while its partner
// reads its next K-tile's fragments from LDS and issues LDS-DMA for the tile
// after — the matrix pipe alternates between the two waves instead of both
// waves reading, then both computing.
//   group 0, K-tile t: [R(t) + DMA(t+1)] bar [M(t) + vmcnt(0)] bar
//   group 1, K-tile t: [M(t-1) + DMA(t+1)] bar [R(t) + vmcnt(0) + lgkmcnt(0)] bar
// DMA(t+1) overwrites buffer (t+1)%2 whose last reader (group 1, slot 2t-1)
// retired its reads before that slot's barrier; K-tile t+1 is waited for by
// every issuing wave before the barrier ending slot 2t+1 and first read in
// slot 2t+2 — both by barrier count, independent of timing.
namespace v3 {
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
}  // namespace v3

template <int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_nt_v3(const half_t* __restrict__ A, const half_t* __restrict__ W,
                                                   half_t* __restrict__ C, int M, int N, int K, int lda, int ldw,
                                                   int ldc, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp_id = wave >> 2;             // ping-pong group (== wm)

  const int nwg = gridDim.x;
  int bid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  }
  const int tiles_m = (M + BM - 1) / BM;
  const int tiles_n = N / BN;
  constexpr int GROUP_M = 8;
  const int group = bid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int in_g = bid - group * GROUP_M * tiles_n;
  const int tm = first_m + in_g % gsz;
  const int tn = in_g / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  // staging pointers: one per-lane base per operand; the 4 pieces of a wave are 8 rows apart
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ lr;
  const half_t* wbase = W + (size_t)(n0 + wave * 32 + lr) * ldw + lc * 8;
  const int xrow0 = m0 + wave * 32 + lr;
  const half_t* xcol = A + lc * 8;
#define V3_STAGE(buf, k0)                                                                 \
  {                                                                                       \
    char* base_ = smem + (buf) * STAGE_BYTES;                                             \
    _Pragma("unroll") for (int j_ = 0; j_ < 4; ++j_)                                      \
      glds16(wbase + (size_t)(j_ * 8) * ldw + (k0), base_ + (wave * 4 + j_) * 1024);      \
    _Pragma("unroll") for (int j_ = 0; j_ < 4; ++j_)                                      \
      glds16(xcol + (size_t)min(xrow0 + j_ * 8, M - 1) * lda + (k0),                      \
             base_ + TILE_BYTES + (wave * 4 + j_) * 1024);                                \
  }

  const int wn = wave & 3, wm = wave >> 2;
  const int fr = lane & 15, grp = lane >> 4;
  const int swz = lane & 7;
  const int wrow = (wn * 64 + fr) * 128;
  const int xrow = TILE_BYTES + (wm * 128 + fr) * 128;
  const int ch0 = ((0 * 4 + grp) ^ swz) << 4;
  const int ch1 = ((1 * 4 + grp) ^ swz) << 4;

  floatx4 acc[8][4];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  half8 wf0[4], wf1[4], xf0[8], xf1[8];   // k-halves 0/1 of the wave's K-tile fragments

#define V3_READ(buf)                                                                      \
  {                                                                                       \
    const char* b_ = smem + (buf) * STAGE_BYTES;                                          \
    _Pragma("unroll") for (int t_ = 0; t_ < 4; ++t_) wf0[t_] = *(const half8*)(b_ + wrow + t_ * 2048 + ch0); \
    _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_) xf0[u_] = *(const half8*)(b_ + xrow + u_ * 2048 + ch0); \
    _Pragma("unroll") for (int t_ = 0; t_ < 4; ++t_) wf1[t_] = *(const half8*)(b_ + wrow + t_ * 2048 + ch1); \
    _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_) xf1[u_] = *(const half8*)(b_ + xrow + u_ * 2048 + ch1); \
  }
#define V3_MMA()                                                                          \
  {                                                                                       \
    __builtin_amdgcn_s_setprio(1);                                                        \
    _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_)                                      \
    _Pragma("unroll") for (int t_ = 0; t_ < 4; ++t_)                                      \
      acc[u_][t_] = mfma16x16x32(wf0[t_], xf0[u_], acc[u_][t_]);                          \
    _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_)                                      \
    _Pragma("unroll") for (int t_ = 0; t_ < 4; ++t_)                                      \
      acc[u_][t_] = mfma16x16x32(wf1[t_], xf1[u_], acc[u_][t_]);                          \
    __builtin_amdgcn_s_setprio(0);                                                        \
  }

  const int nk = K / BK;
  V3_STAGE(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  v3::bar();
  if (grp_id == 0) {
    for (int t = 0; t < nk; ++t) {
      V3_READ(t & 1);
      if (t + 1 < nk) V3_STAGE((t + 1) & 1, (t + 1) * BK);
      v3::bar();
      V3_MMA();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      v3::bar();
    }
  } else {
    for (int t = 0; t < nk; ++t) {
      if (t > 0) V3_MMA();
      if (t + 1 < nk) V3_STAGE((t + 1) & 1, (t + 1) * BK);
      v3::bar();
      V3_READ(t & 1);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      v3::bar();
    }
    V3_MMA();
  }
#undef V3_MMA
#undef V3_READ
#undef V3_STAGE

#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int m = m0 + wm * 128 + u * 16 + fr;
    if (m < M) {
#pragma unroll
      for (int p = 0; p < 2; ++p)
        store_pair<EPI>(C, ldc, m, n0 + wn * 64 + p * 32, grp, acc[u][2 * p], acc[u][2 * p + 1], ep);
    }
  }
}

// ------------------------------------------------------------------ v4
// Latency-hiding ring.  The ablation (scripts/gemm_ablate.py) shows the
// 2-stage loop is bound by LDS-DMA latency: ~64 KiB per CU in flight, ~1.5 us
// per K-step under full-chip load, while MFMA alone would run at 2.2 PF.
// v4 keeps up to 4 BK=32 tiles (128 KiB) in flight in a 5-stage ring that
// uses the whole 160 KiB LDS: tile t+4 is issued while tile t computes and
// the loop only ever waits for tile t+2 (`s_waitcnt vmcnt(8)`, never a
// drain in steady state; raw s_barrier so no implicit vmcnt(0)).
// Fragments are register double-buffered: the ds_reads of tile t+1 are
// issued between the two MFMA halves of tile t.
// LDS image per operand per stage: [256 rows][32 k] fp16 (64-B rows); 16-B
// chunk c of row r stored at c ^ G[(r >> 2) & 3], G = {0,2,3,1}
// (conflict-free for every ds_read_b128 lane group of the fragment read).
namespace v4 {
constexpr int BK4 = 32, NSTAGE = 5;
constexpr int OP_BYTES = 256 * BK4 * 2;      // 16 KiB per operand per stage
constexpr int STAGE4 = 2 * OP_BYTES;          // 32 KiB
constexpr int LDS4 = NSTAGE * STAGE4;         // 160 KiB (the whole CU LDS)
__device__ __forceinline__ int swz_g(int q) { return (0x1320 >> (q * 4)) & 0xF; }
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
}  // namespace v4

template <int EPI, int ABL = 0>
__global__ __launch_bounds__(NT, 2) void gemm_nt_v4(const half_t* __restrict__ A, const half_t* __restrict__ W,
                                                   half_t* __restrict__ C, int M, int N, int K, int lda, int ldw,
                                                   int ldc, Epi ep) {
  using namespace v4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int nwg = gridDim.x;
  int bid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  }
  const int tiles_m = (M + BM - 1) / BM;
  const int tiles_n = N / BN;
  constexpr int GROUP_M = 8;
  const int group = bid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int in_g = bid - group * GROUP_M * tiles_n;
  const int tm = first_m + in_g % gsz;
  const int tn = in_g / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  // staging: a 1 KiB LDS-DMA piece = 16 rows x 64 B; a wave fills 2 pieces per operand per tile
  const int lr = lane >> 2;
  const int lc = (lane & 3) ^ swz_g(lr >> 2);
  const half_t* wbase = W + (size_t)(n0 + wave * 32 + lr) * ldw + lc * 8;
  const int xrow0 = m0 + wave * 32 + lr;
  const half_t* xcol = A + lc * 8;
#define V4_STAGE(st, k0)                                                                  \
  {                                                                                       \
    char* base_ = smem + (st) * STAGE4;                                                   \
    _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_)                                      \
      glds16(wbase + (size_t)(j_ * 16) * ldw + (k0), base_ + (wave * 2 + j_) * 1024);     \
    _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_)                                      \
      glds16(xcol + (size_t)min(xrow0 + j_ * 16, M - 1) * lda + (k0),                     \
             base_ + OP_BYTES + (wave * 2 + j_) * 1024);                                  \
  }

  const int wn = wave & 3, wm = wave >> 2;
  const int fr = lane & 15, grp = lane >> 4;
  const int fch = (grp ^ swz_g(fr >> 2)) << 4;
  const int woff = (wn * 64 + fr) * 64 + fch;
  const int xoff = OP_BYTES + (wm * 128 + fr) * 64 + fch;

  floatx4 acc[8][4];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  half8 wa[4], xa[8], wb[4], xb[8];
  const int nk = K / BK4;   // even (host guarantees), >= 2

#define V4_FRAG_W(st, wf)                                                           \
  {                                                                                 \
    const char* fb_ = smem + (st) * STAGE4 + woff;                                  \
    _Pragma("unroll") for (int t_ = 0; t_ < 4; ++t_) wf[t_] = *(const half8*)(fb_ + t_ * 1024); \
  }
#define V4_FRAG_X(st, xf, h)                                                        \
  {                                                                                 \
    const char* fb_ = smem + (st) * STAGE4 + xoff + (h) * 4096;                     \
    _Pragma("unroll") for (int u_ = 0; u_ < 4; ++u_) xf[(h) * 4 + u_] = *(const half8*)(fb_ + u_ * 1024); \
  }
#define V4_MMA(wf, xf, h)                                                           \
  {                                                                                 \
    __builtin_amdgcn_s_setprio(1);                                                  \
    if (!(ABL & 4)) {                                                               \
    _Pragma("unroll") for (int u_ = 0; u_ < 4; ++u_)                                \
    _Pragma("unroll") for (int t_ = 0; t_ < 4; ++t_)                                \
      acc[(h) * 4 + u_][t_] = mfma16x16x32(wf[t_], xf[(h) * 4 + u_], acc[(h) * 4 + u_][t_]); \
    } else {                                                                        \
    _Pragma("unroll") for (int t_ = 0; t_ < 4; ++t_) asm volatile("" :: "v"(wf[t_])); \
    _Pragma("unroll") for (int u_ = 0; u_ < 4; ++u_) asm volatile("" :: "v"(xf[(h) * 4 + u_])); \
    }                                                                               \
    __builtin_amdgcn_s_setprio(0);                                                  \
  }
  // iteration T: issue tile T+4, compute tile T from (WC, XC) while reading
  // tile T+1 into (WN, XN), then wait until tile T+2 has landed.
#define V4_BODY(T, WC, XC, WN, XN)                                                  \
  {                                                                                 \
    const int t_ = (T);                                                             \
    if (!(ABL & 1) && t_ + 4 < nk) V4_STAGE((t_ + 4) % NSTAGE, (t_ + 4) * BK4);     \
    const int sn_ = (t_ + 1) % NSTAGE;                                              \
    V4_MMA(WC, XC, 0);                                                              \
    __builtin_amdgcn_sched_barrier(0);                                              \
    V4_FRAG_W(sn_, WN);                                                             \
    V4_FRAG_X(sn_, XN, 0);                                                          \
    __builtin_amdgcn_sched_barrier(0);                                              \
    V4_MMA(WC, XC, 1);                                                              \
    __builtin_amdgcn_sched_barrier(0);                                              \
    V4_FRAG_X(sn_, XN, 1);                                                          \
    __builtin_amdgcn_sched_barrier(0);                                              \
    if (t_ + 4 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");               \
    else if (t_ + 3 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");          \
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                           \
    v4::bar();                                                                      \
  }

  // prologue: tiles 0..3 in flight, wait for 0 and 1
  const int pro = nk < 4 ? nk : 4;
  for (int i = 0; i < pro; ++i) V4_STAGE(i, i * BK4);
  if (pro == 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (pro == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  v4::bar();
  V4_FRAG_W(0, wa);
  V4_FRAG_X(0, xa, 0);
  V4_FRAG_X(0, xa, 1);
  if (pro == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (pro == 3) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  v4::bar();
  for (int t = 0; t < nk; t += 2) {
    V4_BODY(t, wa, xa, wb, xb);
    V4_BODY(t + 1, wb, xb, wa, xa);
  }
#undef V4_BODY
#undef V4_MMA
#undef V4_FRAG_X
#undef V4_FRAG_W
#undef V4_STAGE

#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int m = m0 + wm * 128 + u * 16 + fr;
    if (m < M) {
#pragma unroll
      for (int p = 0; p < 2; ++p)
        store_pair<EPI>(C, ldc, m, n0 + wn * 64 + p * 32, grp, acc[u][2 * p], acc[u][2 * p + 1], ep);
    }
  }
}

// ------------------------------------------------------------------ v5
// v1's 2-stage 256x256x64 LDS-DMA loop (whose DMA-only time equals hipBLASLt's
// whole kernel: the L2->LDS stream is the bound, scripts/gemm_ablate.py), with
// the staging work hidden in MFMA issue gaps instead of clustered:
//   * fragments register double-buffered: the 12 ds_reads of k-half 1 are
//     issued inside k-half 0's 32 MFMAs;
//   * the 8 LDS-DMA pieces of tile k+1 are spread 1 per 8 MFMAs;
//   * sched_group_barrier pins the interleave {8 MFMA, 3 DS read, 1 VMEM}.
template <int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_nt_v5(const half_t* __restrict__ A, const half_t* __restrict__ W,
                                                   half_t* __restrict__ C, int M, int N, int K, int lda, int ldw,
                                                   int ldc, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int nwg = gridDim.x;
  int bid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  }
  const int tiles_m = (M + BM - 1) / BM;
  const int tiles_n = N / BN;
  constexpr int GROUP_M = 8;
  const int group = bid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int in_g = bid - group * GROUP_M * tiles_n;
  const int tm = first_m + in_g % gsz;
  const int tn = in_g / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ lr;
  const half_t* wbase = W + (size_t)(n0 + wave * 32 + lr) * ldw + lc * 8;
  const int xrow0 = m0 + wave * 32 + lr;
  const half_t* xcol = A + lc * 8;
  // piece j (0..7): j < 4 -> W rows wave*32 + 8j, else X rows wave*32 + 8(j-4)
#define V5_PIECE(buf, k0, j)                                                              \
  {                                                                                       \
    char* base_ = smem + (buf) * STAGE_BYTES;                                             \
    if ((j) < 4)                                                                          \
      glds16(wbase + (size_t)((j) * 8) * ldw + (k0), base_ + (wave * 4 + (j)) * 1024);    \
    else                                                                                  \
      glds16(xcol + (size_t)min(xrow0 + ((j) - 4) * 8, M - 1) * lda + (k0),               \
             base_ + TILE_BYTES + (wave * 4 + (j) - 4) * 1024);                           \
  }

  const int wn = wave & 3, wm = wave >> 2;
  const int fr = lane & 15, grp = lane >> 4;
  const int swz = lane & 7;
  const int wrow = (wn * 64 + fr) * 128;
  const int xrow = TILE_BYTES + (wm * 128 + fr) * 128;
  const int ch0 = ((0 * 4 + grp) ^ swz) << 4;
  const int ch1 = ((1 * 4 + grp) ^ swz) << 4;

  floatx4 acc[8][4];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  half8 wa[4], xa[8], wb[4], xb[8];

#define V5_READ(buf, ch, wf, xf)                                                          \
  {                                                                                       \
    const char* b_ = smem + (buf) * STAGE_BYTES;                                          \
    _Pragma("unroll") for (int t_ = 0; t_ < 4; ++t_) wf[t_] = *(const half8*)(b_ + wrow + t_ * 2048 + (ch)); \
    _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_) xf[u_] = *(const half8*)(b_ + xrow + u_ * 2048 + (ch)); \
  }
#define V5_MMA(wf, xf)                                                                    \
  {                                                                                       \
    _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_)                                      \
    _Pragma("unroll") for (int t_ = 0; t_ < 4; ++t_)                                      \
      acc[u_][t_] = mfma16x16x32(wf[t_], xf[u_], acc[u_][t_]);                            \
  }

  const int nk = K / BK;
  _Pragma("unroll") for (int j = 0; j < 8; ++j) V5_PIECE(0, 0, j);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  V5_READ(0, ch0, wa, xa);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    // the last iteration re-stages the final tile into the idle buffer (never read):
    // no branch, so each k-half stays one basic block for sched_group_barrier
    const int kn = min(kt + 1, nk - 1) * BK;
    // ---- k-half 0: MFMAs on (wa, xa); read k-half 1 into (wb, xb); 4 DMA pieces
    __builtin_amdgcn_sched_barrier(0);
    V5_READ(cur, ch1, wb, xb);
    V5_PIECE(cur ^ 1, kn, 0) V5_PIECE(cur ^ 1, kn, 1) V5_PIECE(cur ^ 1, kn, 2) V5_PIECE(cur ^ 1, kn, 3)
    V5_MMA(wa, xa);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);   // 8 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);   // 3 DS read
      __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);   // 1 VMEM (LDS-DMA piece)
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- k-half 1: MFMAs on (wb, xb); remaining 4 DMA pieces
    V5_PIECE(cur ^ 1, kn, 4) V5_PIECE(cur ^ 1, kn, 5) V5_PIECE(cur ^ 1, kn, 6) V5_PIECE(cur ^ 1, kn, 7)
    V5_MMA(wb, xb);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    V5_READ(cur ^ 1, ch0, wa, xa);
  }
#undef V5_MMA
#undef V5_READ
#undef V5_PIECE

#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int m = m0 + wm * 128 + u * 16 + fr;
    if (m < M) {
#pragma unroll
      for (int p = 0; p < 2; ++p)
        store_pair<EPI>(C, ldc, m, n0 + wn * 64 + p * 32, grp, acc[u][2 * p], acc[u][2 * p + 1], ep);
    }
  }
}

// ------------------------------------------------------------------ v6
// One wave per SIMD: 4 waves (256 threads) per 256x256x64 block tile, each
// wave owning a 128x128 output quadrant = 8 x 8 tiles of v_mfma_f32_16x16x32_f16
// (256 fp32 accumulators, allocated in AGPRs: launch bounds admit 512
// registers per lane at one wave per SIMD).  Per K-tile a wave issues 128
// MFMAs (2048 matrix-pipe cycles) and only 32 fragment ds_reads (a 128x128
// quadrant re-uses each fragment 8 times — 1/3 fewer LDS reads per FLOP than
// the 8-wave layout) plus 16 LDS-DMA pieces; fragments for the second k-half
// and the next tile's DMA are issued while the current k-half's MFMAs run.
// Same LDS image / swizzle / XCD-aware order as v1.
template <int EPI>
__global__ __launch_bounds__(256, 1) void gemm_nt_v6(const half_t* __restrict__ A, const half_t* __restrict__ W,
                                                    half_t* __restrict__ C, int M, int N, int K, int lda, int ldw,
                                                    int ldc, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int nwg = gridDim.x;
  int bid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  }
  const int tiles_m = (M + BM - 1) / BM;
  const int tiles_n = N / BN;
  constexpr int GROUP_M = 8;
  const int group = bid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int in_g = bid - group * GROUP_M * tiles_n;
  const int tm = first_m + in_g % gsz;
  const int tn = in_g / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  // staging: 32 pieces (1 KiB = 8 rows x 128 B) per operand; a wave fills 8 of each
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ lr;
  const half_t* wbase = W + (size_t)(n0 + wave * 64 + lr) * ldw + lc * 8;
  const int xrow0 = m0 + wave * 64 + lr;
  const half_t* xcol = A + lc * 8;
#define V6_PIECE(buf, k0, j)                                                              \
  {                                                                                       \
    char* base_ = smem + (buf) * STAGE_BYTES;                                             \
    if ((j) < 8)                                                                          \
      glds16(wbase + (size_t)((j) * 8) * ldw + (k0), base_ + (wave * 8 + (j)) * 1024);    \
    else                                                                                  \
      glds16(xcol + (size_t)min(xrow0 + ((j) - 8) * 8, M - 1) * lda + (k0),               \
             base_ + TILE_BYTES + (wave * 8 + (j) - 8) * 1024);                           \
  }

  const int wp = wave & 1, wq = wave >> 1;       // P (W rows) half, Q (X rows) half
  const int fr = lane & 15, grp = lane >> 4;
  const int swz = lane & 7;
  const int wrow = (wp * 128 + fr) * 128;
  const int xrow = TILE_BYTES + (wq * 128 + fr) * 128;
  const int ch0 = ((0 * 4 + grp) ^ swz) << 4;
  const int ch1 = ((1 * 4 + grp) ^ swz) << 4;

  floatx4 acc[8][8];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  half8 wa[8], xa[8], wb[8], xb[8];

#define V6_READ(buf, ch, wf, xf)                                                          \
  {                                                                                       \
    const char* b_ = smem + (buf) * STAGE_BYTES;                                          \
    _Pragma("unroll") for (int t_ = 0; t_ < 8; ++t_) wf[t_] = *(const half8*)(b_ + wrow + t_ * 2048 + (ch)); \
    _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_) xf[u_] = *(const half8*)(b_ + xrow + u_ * 2048 + (ch)); \
  }
#define V6_MMA(wf, xf)                                                                    \
  {                                                                                       \
    _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_)                                      \
    _Pragma("unroll") for (int t_ = 0; t_ < 8; ++t_)                                      \
      acc[u_][t_] = mfma16x16x32(wf[t_], xf[u_], acc[u_][t_]);                            \
  }

  const int nk = K / BK;
  _Pragma("unroll") for (int j = 0; j < 16; ++j) V6_PIECE(0, 0, j);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  V6_READ(0, ch0, wa, xa);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const int kn = min(kt + 1, nk - 1) * BK;    // last iteration re-stages into the idle buffer
    __builtin_amdgcn_sched_barrier(0);
    // ---- k-half 0 (64 MFMAs): first the k-half-1 fragments from `cur`, then
    // the next tile's 16 DMA pieces into `cur^1` (reads before writes: the
    // compiler must assume the LDS accesses alias, so this order lets it interleave)
    V6_READ(cur, ch1, wb, xb);
    _Pragma("unroll") for (int j = 0; j < 16; ++j) V6_PIECE(cur ^ 1, kn, j);
    V6_MMA(wa, xa);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // 4 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);   // 4 DS read
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);   // 3 MFMA
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // 1 VMEM read (LDS-DMA piece)
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- k-half 1: 32 MFMAs, then wait for the DMA + barrier (every wave is
    // done reading `cur`, so the next iteration may overwrite it), then the
    // next tile's k-half-0 fragments are read under the remaining 32 MFMAs.
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[u][t] = mfma16x16x32(wb[t], xb[u], acc[u][t]);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    V6_READ(cur ^ 1, ch0, wa, xa);
#pragma unroll
    for (int u = 4; u < 8; ++u)
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[u][t] = mfma16x16x32(wb[t], xb[u], acc[u][t]);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // 4 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // 2 DS read
    }
  }
#undef V6_MMA
#undef V6_READ
#undef V6_PIECE

#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int m = m0 + wq * 128 + u * 16 + fr;
    if (m < M) {
#pragma unroll
      for (int p = 0; p < 4; ++p)
        store_pair<EPI>(C, ldc, m, n0 + wp * 128 + p * 32, grp, acc[u][2 * p], acc[u][2 * p + 1], ep);
    }
  }
}

int g_variant = -1;   // -1: from env FLS_GEMM_VARIANT (default 3)

int variant() {
  if (g_variant < 0) {
    const char* e = getenv("FLS_GEMM_VARIANT");
    g_variant = e ? atoi(e) : 3;
  }
  return g_variant;
}

template <int EPI>
int launch(const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda, int ldw, int ldc,
           const Epi& ep, hipStream_t s) {
  const int var = variant();
  const bool fast = (N % BN == 0) && (K % BK == 0) && (lda % 8 == 0) && (ldw % 8 == 0) && M > 0;
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  const bool fast4 = fast && (K % (2 * v4::BK4) == 0);
  if (var == 6 && fast) {
    static bool attr6 = false;
    if (!attr6) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_v6<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
      attr6 = true;
    }
    hipLaunchKernelGGL(gemm_nt_v6<EPI>, dim3(tiles), dim3(256), LDS_BYTES, s, A, W, C, M, N, K, lda, ldw, ldc, ep);
  } else if (var == 5 && fast) {
    static bool attr5 = false;
    if (!attr5) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_v5<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
      attr5 = true;
    }
    hipLaunchKernelGGL(gemm_nt_v5<EPI>, dim3(tiles), dim3(NT), LDS_BYTES, s, A, W, C, M, N, K, lda, ldw, ldc, ep);
  } else if (var == 4 && fast4) {
    static bool attr4 = false;
    if (!attr4) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_v4<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, v4::LDS4);
      attr4 = true;
    }
    hipLaunchKernelGGL(gemm_nt_v4<EPI>, dim3(tiles), dim3(NT), v4::LDS4, s, A, W, C, M, N, K, lda, ldw, ldc, ep);
  } else if (var == 3 && fast) {
    static bool attr3 = false;
    if (!attr3) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_v3<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
      attr3 = true;
    }
    hipLaunchKernelGGL(gemm_nt_v3<EPI>, dim3(tiles), dim3(NT), LDS_BYTES, s, A, W, C, M, N, K, lda, ldw, ldc, ep);
  } else if (var >= 1 && fast) {
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_256x256<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
      attr_set = true;
    }
    hipLaunchKernelGGL(gemm_nt_256x256<EPI>, dim3(tiles), dim3(NT), LDS_BYTES, s, A, W, C, M, N, K, lda, ldw, ldc, ep);
  } else {
    dim3 grid((M + 31) / 32, (N + 255) / 256);
    hipLaunchKernelGGL(gemm_nt_generic<EPI>, grid, dim3(256), 0, s, A, W, C, M, N, K, lda, ldw, ldc, ep);
  }
  FLS_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int fls_kernels_version(void) { return 2; }

// microbenchmark-only entry: v1 main loop with parts removed (results are garbage)
extern "C" int fls_gemm_ablate(int abl, const void* A, const void* W, void* C, int M, int N, int K,
                               fls_stream_t s) {
  if (N % BN || K % BK) return -2;
  Epi ep{nullptr, 0, nullptr, nullptr, nullptr, 0, 0};
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  auto a = (const half_t*)A;
  auto w = (const half_t*)W;
  auto c = (half_t*)C;
#define FLS_ABL_CASE(X)                                                                                      \
  case X:                                                                                                    \
    (void)hipFuncSetAttribute((const void*)gemm_nt_256x256<0, X>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                              LDS_BYTES);                                                                   \
    hipLaunchKernelGGL((gemm_nt_256x256<0, X>), dim3(tiles), dim3(NT), LDS_BYTES, (hipStream_t)s, a, w, c, M, N, K, \
                       K, K, N, ep);                                                                         \
    break;
#define FLS_ABL4_CASE(X)                                                                                     \
  case 10 + X:                                                                                               \
    (void)hipFuncSetAttribute((const void*)gemm_nt_v4<0, X>, hipFuncAttributeMaxDynamicSharedMemorySize,     \
                              v4::LDS4);                                                                     \
    hipLaunchKernelGGL((gemm_nt_v4<0, X>), dim3(tiles), dim3(NT), v4::LDS4, (hipStream_t)s, a, w, c, M, N, K, \
                       K, K, N, ep);                                                                         \
    break;
  switch (abl) {
    FLS_ABL_CASE(0) FLS_ABL_CASE(1) FLS_ABL_CASE(2) FLS_ABL_CASE(3) FLS_ABL_CASE(4) FLS_ABL_CASE(5) FLS_ABL_CASE(6)
    FLS_ABL4_CASE(0) FLS_ABL4_CASE(1) FLS_ABL4_CASE(4)
    case 20:
      (void)hipFuncSetAttribute((const void*)gemm_nt_256x256<0, 0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                LDS_BYTES);
      hipLaunchKernelGGL((gemm_nt_256x256<0, 0, 1>), dim3(tiles), dim3(NT), LDS_BYTES, (hipStream_t)s, a, w, c, M, N,
                         K, K, K, N, ep);
      break;
    case 26:
      (void)hipFuncSetAttribute((const void*)gemm_nt_256x256<0, 6, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                LDS_BYTES);
      hipLaunchKernelGGL((gemm_nt_256x256<0, 6, 1>), dim3(tiles), dim3(NT), LDS_BYTES, (hipStream_t)s, a, w, c, M, N,
                         K, K, K, N, ep);
      break;
    default: return -3;
  }
#undef FLS_ABL4_CASE
#undef FLS_ABL_CASE
  FLS_CHECK_LAUNCH();
  return 0;
}

// select the GEMM main-loop variant (0 generic, 1 = 256x256x64 2-stage, 3 = ping-pong 2-stage)
extern "C" int fls_gemm_set_variant(int v) {
  const int old = variant();
  g_variant = v;
  return old;
}

extern "C" int fls_gemm(const void* A, const void* W, void* C, const void* R, int M, int N, int K, int lda, int ldw,
                        int ldc, int ldr, int epi, const int* pos, const float* cos_t, const float* sin_t,
                        int rope_cols, int head_dim, fls_stream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if ((epi == FLS_EPI_SWIGLU || epi == FLS_EPI_ROPE) && (N % 32)) return -2;
  if (epi == FLS_EPI_ROPE && (head_dim % 32 || rope_cols % 32)) return -3;
  Epi ep{(const half_t*)R, ldr, pos, cos_t, sin_t, rope_cols, head_dim};
  auto a = (const half_t*)A;
  auto w = (const half_t*)W;
  auto c = (half_t*)C;
  auto st = (hipStream_t)s;
  switch (epi) {
    case FLS_EPI_NONE: return launch<FLS_EPI_NONE>(a, w, c, M, N, K, lda, ldw, ldc, ep, st);
    case FLS_EPI_RESID: return launch<FLS_EPI_RESID>(a, w, c, M, N, K, lda, ldw, ldc, ep, st);
    case FLS_EPI_SWIGLU: return launch<FLS_EPI_SWIGLU>(a, w, c, M, N, K, lda, ldw, ldc, ep, st);
    case FLS_EPI_ROPE: return launch<FLS_EPI_ROPE>(a, w, c, M, N, K, lda, ldw, ldc, ep, st);
  }
  return -1;
}
