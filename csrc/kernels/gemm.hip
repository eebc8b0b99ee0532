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
  const half_t* bias;   // optional per-output-column bias (Qwen2 q/k/v, Llama attention_bias), added first
};

// Store one pair of 16-column subtiles (cols n_first + 4*grp + r and +16)
// for output row m.  acc_a: first subtile, acc_b: second (its partner).
// n_first: first column of the 32-column block (gate|up or rotation-pair block);
// off: the lane's 4-column group inside its first 16 columns (acc_b is 16 columns on).
template <int EPI>
__device__ __forceinline__ void store_pair_off(half_t* __restrict__ C, int ldc, int m, int n_first, int off,
                                               const floatx4& acc_a, const floatx4& acc_b, const Epi& ep) {
  const int c0 = n_first + off;
  if constexpr (EPI == FLS_EPI_SWIGLU) {
    // pair = (gate, up) of intermediate columns [n_first/2, n_first/2 + 16)
    const int oc = n_first / 2 + off;
    half4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (half_t)(silu(acc_a[r]) * acc_b[r]);
    *(half4*)(C + (size_t)m * ldc + oc) = o;
    return;
  } else {
    floatx4 a = acc_a, b = acc_b;
    if (ep.bias) {
      const half4 ba = *(const half4*)(ep.bias + c0);
      const half4 bb = *(const half4*)(ep.bias + c0 + 16);
#pragma unroll
      for (int r = 0; r < 4; ++r) { a[r] += (float)ba[r]; b[r] += (float)bb[r]; }
    }
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
          const float x1 = a[r], x2 = b[r];
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

template <int EPI>
__device__ __forceinline__ void store_pair(half_t* __restrict__ C, int ldc, int m, int n_first, int grp,
                                           const floatx4& acc_a, const floatx4& acc_b, const Epi& ep) {
  store_pair_off<EPI>(C, ldc, m, n_first, 4 * grp, acc_a, acc_b, ep);
}

// Epilogue of a wave's 128 (M) x 128 (N) quadrant held as acc[8 row groups][8 subtiles] (v10).
// store_pair issues each row's operand loads (residual rows, RoPE position + cos/sin) right
// before that row's stores, and because R may alias C the compiler cannot hoist the next
// row's loads above them: 8 dependent load -> store round trips per tile while the matrix
// pipe idles (scripts/gemm_epi_cost.py: RoPE cost 8% of the 70B QKV GEMM, 15% at K = 4096).
// Here row group u+1's loads are issued before row group u's stores (different rows, so
// in-place R == C stays correct), the positions of all 8 row groups are loaded up front and
// the per-column bias once.
template <int EPI>
__device__ __forceinline__ void epilogue_quadrant(half_t* __restrict__ C, int ldc, int M, int mrow0, int ncol0,
                                                  int grp, floatx4 (&acc)[8][8], const Epi& ep) {
  const int off = 4 * grp;
  if constexpr (EPI == FLS_EPI_NONE || EPI == FLS_EPI_SWIGLU) {
    if (EPI == FLS_EPI_SWIGLU || ep.bias == nullptr) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int m = mrow0 + u * 16;
        if (m < M) {
#pragma unroll
          for (int p = 0; p < 4; ++p)
            store_pair_off<EPI>(C, ldc, m, ncol0 + p * 32, off, acc[u][2 * p], acc[u][2 * p + 1], ep);
        }
      }
      return;
    }
  }
  // per-column bias (same for every row): once, kept as fp16
  half4 ba[4], bb[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (ep.bias) {
      ba[p] = *(const half4*)(ep.bias + ncol0 + p * 32 + off);
      bb[p] = *(const half4*)(ep.bias + ncol0 + p * 32 + off + 16);
    } else {
      ba[p] = half4{0, 0, 0, 0};
      bb[p] = half4{0, 0, 0, 0};
    }
  }
  if constexpr (EPI == FLS_EPI_RESID) {
    half4 ra[2][4], rb[2][4];
    auto load = [&](int u, int sl) {
      const int m = min(mrow0 + u * 16, M - 1);
      const half_t* rp = ep.R + (size_t)m * ep.ldr + ncol0 + off;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        ra[sl][p] = *(const half4*)(rp + p * 32);
        rb[sl][p] = *(const half4*)(rp + p * 32 + 16);
      }
    };
    load(0, 0);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int sl = u & 1;
      if (u + 1 < 8) load(u + 1, sl ^ 1);
      // keep the loads exactly one row group ahead: the cos/sin tables (float) cannot alias C
      // (half), so without a fence the compiler hoists all 8 rows' loads and spills
      asm volatile("" ::: "memory");
      const int m = mrow0 + u * 16;
      if (m < M) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          half4 oa, ob;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            oa[r] = (half_t)(acc[u][2 * p][r] + (float)ba[p][r] + (float)ra[sl][p][r]);
            ob[r] = (half_t)(acc[u][2 * p + 1][r] + (float)bb[p][r] + (float)rb[sl][p][r]);
          }
          half_t* cp = C + (size_t)m * ldc + ncol0 + p * 32 + off;
          *(half4*)cp = oa;
          *(half4*)(cp + 16) = ob;
        }
      }
    }
  } else if constexpr (EPI == FLS_EPI_ROPE) {
    const int hd = ep.head_dim, half_hd = hd >> 1;
    int pos[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) pos[u] = ep.pos[min(mrow0 + u * 16, M - 1)];
    int f0[4];
    bool rot[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int o = (ncol0 + p * 32 + off) % hd;
      f0[p] = (o >> 5) * 16 + (o & 15);
      rot[p] = ncol0 + p * 32 < ep.rope_cols;       // wave-uniform
    }
    floatx4 cs[2][4], sn[2][4];
    auto load = [&](int u, int sl) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        if (rot[p]) {
          cs[sl][p] = *(const floatx4*)(ep.cos_t + (size_t)pos[u] * half_hd + f0[p]);
          sn[sl][p] = *(const floatx4*)(ep.sin_t + (size_t)pos[u] * half_hd + f0[p]);
        }
      }
    };
    load(0, 0);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int sl = u & 1;
      if (u + 1 < 8) load(u + 1, sl ^ 1);
      // keep the loads exactly one row group ahead: the cos/sin tables (float) cannot alias C
      // (half), so without a fence the compiler hoists all 8 rows' loads and spills
      asm volatile("" ::: "memory");
      const int m = mrow0 + u * 16;
      if (m < M) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          half4 oa, ob;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x1 = acc[u][2 * p][r] + (float)ba[p][r], x2 = acc[u][2 * p + 1][r] + (float)bb[p][r];
            if (rot[p]) {
              const float c = cs[sl][p][r], sv = sn[sl][p][r];
              const float y1 = x1 * c - x2 * sv, y2 = x2 * c + x1 * sv;
              x1 = y1;
              x2 = y2;
            }
            oa[r] = (half_t)x1;
            ob[r] = (half_t)x2;
          }
          half_t* cp = C + (size_t)m * ldc + ncol0 + p * 32 + off;
          *(half4*)cp = oa;
          *(half4*)(cp + 16) = ob;
        }
      }
    }
  } else {   // NONE with bias
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int m = mrow0 + u * 16;
      if (m < M) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          half4 oa, ob;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            oa[r] = (half_t)(acc[u][2 * p][r] + (float)ba[p][r]);
            ob[r] = (half_t)(acc[u][2 * p + 1][r] + (float)bb[p][r]);
          }
          half_t* cp = C + (size_t)m * ldc + ncol0 + p * 32 + off;
          *(half4*)cp = oa;
          *(half4*)(cp + 16) = ob;
        }
      }
    }
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
              if (ep.bias) v += (float)ep.bias[n];
              if constexpr (EPI == FLS_EPI_RESID) v += (float)ep.R[(size_t)m * ep.ldr + n];
              C[(size_t)m * ldc + n] = (half_t)v;
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
// Same C^T fragment orientation and epilogues as the main kernels.
namespace mid {
constexpr int BMm = 64, BNm = 128, BKm = 64, NTm = 256, NSTAGE = 3;
constexpr int STAGE = (BMm + BNm) * BKm * 2;     // 24 KiB: A rows 0..63 then W rows 0..127
constexpr int GROUPS = (BMm + BNm) / 8;          // 8-row (1 KiB) LDS-DMA groups per stage
constexpr int PER_WAVE = GROUPS / 4;             // 6 LDS-DMA per wave per stage
}  // namespace mid

template <int EPI>
__global__ __launch_bounds__(mid::NTm) void gemm_nt_mid(const half_t* __restrict__ A, const half_t* __restrict__ W,
                                                     half_t* __restrict__ C, int M, int N, int K, int lda, int ldw,
                                                     int ldc, Epi ep) {
  using namespace mid;
  extern __shared__ __attribute__((aligned(16))) char lds_mid[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, grp = lane >> 4;
  const int mt = (M + BMm - 1) / BMm, ntn = N / BNm;
  // XCD-aware bijective remap: logical tiles [xcd*q .. ) run on one XCD, M fastest
  int bid = blockIdx.x;
  {
    const int nwg = mt * ntn;
    const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    if (nwg >= 8) bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  }
  const int m0 = (bid % mt) * BMm;
  const int n0 = (bid / mt) * BNm;
  const int wm = wave >> 1, wn = wave & 1;
  const int nk = K / BKm;

  // this lane's LDS-DMA sources: group g = wave + 4*i covers tile rows 8*g .. 8*g+7
  const half_t* src[PER_WAVE];
  const int sub = lane >> 3;                       // row inside the 8-row group
  const int kc = ((lane & 7) ^ sub) * 8;           // source chunk pre-swizzled (read XORs it back)
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int g = wave + 4 * i;
    if (g < BMm / 8) {
      const int m = min(m0 + g * 8 + sub, M - 1);
      src[i] = A + (size_t)m * lda + kc;
    } else {
      const int n = n0 + (g - BMm / 8) * 8 + sub;
      src[i] = W + (size_t)n * ldw + kc;
    }
  }
  auto stage = [&](int kt) {
    char* base = lds_mid + (kt % NSTAGE) * STAGE;
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) glds16(src[i] + (size_t)kt * BKm, base + (wave + 4 * i) * 1024);
  };

  floatx4 acc[2][4];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};

  stage(0);
  if (nk > 1) stage(1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 2 < nk) {
      stage(kt + 2);
      asm volatile("s_waitcnt vmcnt(12)" ::: "memory");   // tiles kt+1, kt+2 stay in flight
    } else if (kt + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();                          // every wave's part of tile kt landed
    const char* Xs = lds_mid + (kt % NSTAGE) * STAGE;
    const char* Ws = Xs + BMm * BKm * 2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + grp;                          // logical 16-byte chunk of this lane
      half8 xf[2], wf[4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r = wm * 32 + u * 16 + fr;
        xf[u] = *(const half8*)(Xs + r * 128 + ((c ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int r = wn * 64 + t * 16 + fr;
        wf[t] = *(const half8*)(Ws + r * 128 + ((c ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[u][t] = mfma16x16x32(wf[t], xf[u], acc[u][t]);
    }
    // WAR: stage(kt + 3) (next iteration) overwrites this buffer; all reads are done
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int m = m0 + wm * 32 + u * 16 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int p = 0; p < 2; ++p)
      store_pair<EPI>(C, ldc, m, n0 + wn * 64 + p * 32, grp, acc[u][2 * p], acc[u][2 * p + 1], ep);
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

// ------------------------------------------------------------------ v7
// 8 waves (2 M x 4 N, 128x64 outputs each), 256x256x64 tiles, 4 phases per
// K-tile; each phase = {fragment ds_reads || one half-tile LDS-DMA} ->
// barrier -> lgkmcnt(0) -> 16 MFMAs (one 64x32 C-quadrant x K=64, at raised
// priority) -> barrier.  The four half-tiles of a stage are the row sets the
// phases read, so each is re-filled as soon as its last reader has passed a
// barrier:
//   XA = X rows {0-63, 128-191}  (read phase 0)   XB = X rows {64-127, 192-255} (phase 2)
//   WA = W rows {64w + 0..31}    (read phase 0)   WB = W rows {64w + 32..63}    (phase 1)
// Issue order per K-tile t: ph0 XB(t+1) -> buf t+1; ph1 XA(t+2), ph2 WA(t+2),
// ph3 WB(t+2) -> buf t (their regions were consumed in this tile).  One
// counted `vmcnt(6)` (3 half-tiles x 2 pieces left in flight) before phase
// 3's first barrier retires everything tile t+1 reads; no vmcnt(0) in the
// loop, so staging latency overlaps ~1.5 K-tiles of MFMA work.
// Out-of-range prefetches are clamped to the last K-tile (harmless re-loads into
// consumed regions) so the wait count is uniform.
namespace v7 {
constexpr int BUF = 65536;        // one stage: X image 32 KiB + W image 32 KiB
constexpr int WIMG = 32768;
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_nt_v7(const half_t* __restrict__ A, const half_t* __restrict__ W,
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

  // ---- staging: each wave moves pieces j = 2*wave, 2*wave+1 (8 rows x 128 B) of a half-tile
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ lr;              // source-side XOR swizzle (LDS image stays lane-linear)
  const int j0 = 2 * wave, j1 = 2 * wave + 1;
  const int xr0 = (j0 >> 3) * 128 + (j0 & 7) * 8, xr1 = (j1 >> 3) * 128 + (j1 & 7) * 8;   // XA rows; XB = +64
  const int wr0 = (j0 >> 2) * 64 + (j0 & 3) * 8, wr1 = (j1 >> 2) * 64 + (j1 & 3) * 8;     // WA rows; WB = +32
  const half_t* xa0 = A + (size_t)min(m0 + xr0 + lr, M - 1) * lda + lc * 8;
  const half_t* xa1 = A + (size_t)min(m0 + xr1 + lr, M - 1) * lda + lc * 8;
  const half_t* xb0 = A + (size_t)min(m0 + xr0 + 64 + lr, M - 1) * lda + lc * 8;
  const half_t* xb1 = A + (size_t)min(m0 + xr1 + 64 + lr, M - 1) * lda + lc * 8;
  const half_t* wa0 = W + (size_t)(n0 + wr0 + lr) * ldw + lc * 8;
  const half_t* wa1 = W + (size_t)(n0 + wr1 + lr) * ldw + lc * 8;
  const size_t wb_off = (size_t)32 * ldw;
#define V7_XA(buf, k0) { glds16(xa0 + (k0), smem + (buf) * v7::BUF + xr0 * 128); \
                         glds16(xa1 + (k0), smem + (buf) * v7::BUF + xr1 * 128); }
#define V7_XB(buf, k0) { glds16(xb0 + (k0), smem + (buf) * v7::BUF + (xr0 + 64) * 128); \
                         glds16(xb1 + (k0), smem + (buf) * v7::BUF + (xr1 + 64) * 128); }
#define V7_WA(buf, k0) { glds16(wa0 + (k0), smem + (buf) * v7::BUF + v7::WIMG + wr0 * 128); \
                         glds16(wa1 + (k0), smem + (buf) * v7::BUF + v7::WIMG + wr1 * 128); }
#define V7_WB(buf, k0) { glds16(wa0 + wb_off + (k0), smem + (buf) * v7::BUF + v7::WIMG + (wr0 + 32) * 128); \
                         glds16(wa1 + wb_off + (k0), smem + (buf) * v7::BUF + v7::WIMG + (wr1 + 32) * 128); }

  // ---- fragments: lane (fr, grp) reads row fr of a 16-row fragment, k chunk s*4+grp
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, grp = lane >> 4;
  const int sw = fr & 7;
  const int c0 = ((0 + grp) ^ sw) << 4;         // k-step 0 chunk
  const int c1 = ((4 + grp) ^ sw) << 4;         // k-step 1 chunk
  const int xrow = (wm * 128 + fr) * 128;
  const int wrow = v7::WIMG + (wn * 64 + fr) * 128;

  floatx4 acc[8][4];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  half8 xf[8][2], wf[4][2];

#define V7_RX(buf, u0)                                                                              \
  _Pragma("unroll") for (int u_ = (u0); u_ < (u0) + 4; ++u_) {                                      \
    xf[u_][0] = *(const half8*)(smem + (buf) * v7::BUF + xrow + u_ * 2048 + c0);                    \
    xf[u_][1] = *(const half8*)(smem + (buf) * v7::BUF + xrow + u_ * 2048 + c1);                    \
  }
#define V7_RW(buf, t0)                                                                              \
  _Pragma("unroll") for (int t_ = (t0); t_ < (t0) + 2; ++t_) {                                      \
    wf[t_][0] = *(const half8*)(smem + (buf) * v7::BUF + wrow + t_ * 2048 + c0);                    \
    wf[t_][1] = *(const half8*)(smem + (buf) * v7::BUF + wrow + t_ * 2048 + c1);                    \
  }
#define V7_MMA(u0, t0)                                                                              \
  {                                                                                                 \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                              \
    __builtin_amdgcn_s_setprio(1);                                                                  \
    _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                                \
    _Pragma("unroll") for (int u_ = (u0); u_ < (u0) + 4; ++u_)                                      \
    _Pragma("unroll") for (int t_ = (t0); t_ < (t0) + 2; ++t_)                                      \
      acc[u_][t_] = mfma16x16x32(wf[t_][s_], xf[u_][s_], acc[u_][t_]);                              \
    __builtin_amdgcn_s_setprio(0);                                                                  \
  }

  const int nk = K / BK;
  const int k1p = min(1, nk - 1) * BK;
  V7_XA(0, 0); V7_WA(0, 0); V7_WB(0, 0); V7_XB(0, 0);
  V7_XA(1, k1p); V7_WA(1, k1p); V7_WB(1, k1p);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const int k1 = min(kt + 1, nk - 1) * BK;
    const int k2 = min(kt + 2, nk - 1) * BK;
    // phase 0: read X-half0 + W-half0; stage XB(t+1)
    V7_RX(cur, 0); V7_RW(cur, 0);
    V7_XB(cur ^ 1, k1);
    __builtin_amdgcn_s_barrier();
    V7_MMA(0, 0);
    __builtin_amdgcn_s_barrier();
    // phase 1: read W-half1; stage XA(t+2)
    V7_RW(cur, 2);
    V7_XA(cur, k2);
    __builtin_amdgcn_s_barrier();
    V7_MMA(0, 2);
    __builtin_amdgcn_s_barrier();
    // phase 2: read X-half1; stage WA(t+2)
    V7_RX(cur, 4);
    V7_WA(cur, k2);
    __builtin_amdgcn_s_barrier();
    V7_MMA(4, 2);
    __builtin_amdgcn_s_barrier();
    // phase 3: stage WB(t+2); retire everything tile t+1 reads
    V7_WB(cur, k2);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    V7_MMA(4, 0);
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the block exits
#undef V7_MMA
#undef V7_RW
#undef V7_RX
#undef V7_WB
#undef V7_WA
#undef V7_XB
#undef V7_XA

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

// ------------------------------------------------------------------ v8
// v7's tile/wave geometry with the fragment reads moved ONE PHASE AHEAD of
// the MFMAs that use them, so LDS read latency hides behind a phase of MFMA
// work instead of being exposed before it.  This works without extra
// registers because the quadrant order alternates with tile parity:
//   even tile: (x0,w0) (x0,w1) (x1,w1) (x1,w0)    odd tile: (x0,w1) (x0,w0) (x1,w0) (x1,w1)
// so in every phase exactly one fragment half (4 or 8 ds_read_b128) is free
// and is refilled for a later phase:
//   even t: ph0 w1(t)  ph1 x1(t)  ph2 x0(t+1)  ph3 w1(t+1)
//   odd t:  ph0 w0(t)  ph1 x1(t)  ph2 x0(t+1)  ph3 w0(t+1)
// Half-tile k of tile t+2 is DMA'd in phase k of tile t (XA, W-first, W-second,
// XB), each exactly 6 phases before its first read; per phase:
//   lgkmcnt(0) -> ds_reads (next) -> 2 glds -> vmcnt(10) -> s_barrier -> 16 MFMA
// One barrier per phase covers both hazards: RAW (every wave's counted vmcnt
// precedes the barrier before the read) and WAR (a region is refilled >= 2
// phases after its reads were issued, i.e. after a barrier that follows their
// lgkmcnt(0)).  Up to 6 half-tiles (96 KiB) of staging are in flight per CU.
// Requires an even number of K-tiles (2-tile unrolled body).
template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_nt_v8(const half_t* __restrict__ A, const half_t* __restrict__ W,
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
  const int j0 = 2 * wave, j1 = 2 * wave + 1;
  const int xr0 = (j0 >> 3) * 128 + (j0 & 7) * 8, xr1 = (j1 >> 3) * 128 + (j1 & 7) * 8;
  const int wr0 = (j0 >> 2) * 64 + (j0 & 3) * 8, wr1 = (j1 >> 2) * 64 + (j1 & 3) * 8;
  const half_t* xa0 = A + (size_t)min(m0 + xr0 + lr, M - 1) * lda + lc * 8;
  const half_t* xa1 = A + (size_t)min(m0 + xr1 + lr, M - 1) * lda + lc * 8;
  const half_t* xb0 = A + (size_t)min(m0 + xr0 + 64 + lr, M - 1) * lda + lc * 8;
  const half_t* xb1 = A + (size_t)min(m0 + xr1 + 64 + lr, M - 1) * lda + lc * 8;
  const half_t* wa0 = W + (size_t)(n0 + wr0 + lr) * ldw + lc * 8;
  const half_t* wa1 = W + (size_t)(n0 + wr1 + lr) * ldw + lc * 8;
  const size_t wb_off = (size_t)32 * ldw;
#define V8_XA(buf, k0) { glds16(xa0 + (k0), smem + (buf) * v7::BUF + xr0 * 128); \
                         glds16(xa1 + (k0), smem + (buf) * v7::BUF + xr1 * 128); }
#define V8_XB(buf, k0) { glds16(xb0 + (k0), smem + (buf) * v7::BUF + (xr0 + 64) * 128); \
                         glds16(xb1 + (k0), smem + (buf) * v7::BUF + (xr1 + 64) * 128); }
#define V8_WA(buf, k0) { glds16(wa0 + (k0), smem + (buf) * v7::BUF + v7::WIMG + wr0 * 128); \
                         glds16(wa1 + (k0), smem + (buf) * v7::BUF + v7::WIMG + wr1 * 128); }
#define V8_WB(buf, k0) { glds16(wa0 + wb_off + (k0), smem + (buf) * v7::BUF + v7::WIMG + (wr0 + 32) * 128); \
                         glds16(wa1 + wb_off + (k0), smem + (buf) * v7::BUF + v7::WIMG + (wr1 + 32) * 128); }

  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, grp = lane >> 4;
  const int sw = fr & 7;
  const int c0 = ((0 + grp) ^ sw) << 4;
  const int c1 = ((4 + grp) ^ sw) << 4;
  const int xrow = (wm * 128 + fr) * 128;
  const int wrow = v7::WIMG + (wn * 64 + fr) * 128;

  floatx4 acc[8][4];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  half8 xf[8][2], wf[4][2];

#define V8_RX(buf, h)                                                                               \
  _Pragma("unroll") for (int u_ = (h) * 4; u_ < (h) * 4 + 4; ++u_) {                                \
    xf[u_][0] = *(const half8*)(smem + (buf) * v7::BUF + xrow + u_ * 2048 + c0);                    \
    xf[u_][1] = *(const half8*)(smem + (buf) * v7::BUF + xrow + u_ * 2048 + c1);                    \
  }
#define V8_RW(buf, h)                                                                               \
  _Pragma("unroll") for (int t_ = (h) * 2; t_ < (h) * 2 + 2; ++t_) {                                \
    wf[t_][0] = *(const half8*)(smem + (buf) * v7::BUF + wrow + t_ * 2048 + c0);                    \
    wf[t_][1] = *(const half8*)(smem + (buf) * v7::BUF + wrow + t_ * 2048 + c1);                    \
  }
#define V8_PHASE(xh, wh, READ, DMA)                                                                 \
  {                                                                                                 \
    __builtin_amdgcn_s_waitcnt(0xC07F);     /* lgkmcnt(0), visible to the waitcnt pass */          \
    READ;                                                                                           \
    DMA;                                                                                            \
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");                                               \
    __builtin_amdgcn_s_barrier();                                                                   \
    __builtin_amdgcn_s_setprio(1);                                                                  \
    _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                                \
    _Pragma("unroll") for (int u_ = (xh) * 4; u_ < (xh) * 4 + 4; ++u_)                              \
    _Pragma("unroll") for (int t_ = (wh) * 2; t_ < (wh) * 2 + 2; ++t_)                              \
      acc[u_][t_] = mfma16x16x32(wf[t_][s_], xf[u_][s_], acc[u_][t_]);                              \
    __builtin_amdgcn_s_setprio(0);                                                                  \
  }

  const int nk = K / BK;                       // even (host-checked)
  // prologue = virtual phases -8..-1: tile 0 -> buf 0 (XA, WA, WB, XB), tile 1 -> buf 1 (XA, WB, WA, XB)
  V8_XA(0, 0); V8_WA(0, 0); V8_WB(0, 0); V8_XB(0, 0);
  V8_XA(1, BK); V8_WB(1, BK); V8_WA(1, BK); V8_XB(1, BK);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  V8_RX(0, 0); V8_RW(0, 0);                    // x0(0), w0(0): tile 0's first quadrant
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; kt += 2) {
    const int ka = min(kt + 2, nk - 1) * BK;   // tile kt+2 -> buf 0
    const int kb = min(kt + 3, nk - 1) * BK;   // tile kt+3 -> buf 1
    // even tile kt (buf 0)
    V8_PHASE(0, 0, V8_RW(0, 1), V8_XA(0, ka));
    V8_PHASE(0, 1, V8_RX(0, 1), V8_WA(0, ka));
    V8_PHASE(1, 1, V8_RX(1, 0), V8_WB(0, ka));
    V8_PHASE(1, 0, V8_RW(1, 1), V8_XB(0, ka));
    // odd tile kt+1 (buf 1)
    V8_PHASE(0, 1, V8_RW(1, 0), V8_XA(1, kb));
    V8_PHASE(0, 0, V8_RX(1, 1), V8_WB(1, kb));
    V8_PHASE(1, 0, V8_RX(0, 0), V8_WA(1, kb));
    V8_PHASE(1, 1, V8_RW(0, 0), V8_XB(1, kb));
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#undef V8_PHASE
#undef V8_RW
#undef V8_RX
#undef V8_WB
#undef V8_WA
#undef V8_XB
#undef V8_XA

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

// ------------------------------------------------------------------ v9
// v6's geometry (4 waves = one per SIMD, 128x128 outputs per wave in 256
// AGPR accumulators: 2/3 of the LDS fragment reads per FLOP of the 8-wave
// kernels) with v8's read-ahead schedule, and the LDS reads and DMA
// interleaved INTO the MFMA stream (one wave per SIMD: nothing else would
// fill the matrix pipe while they issue).  Per phase (one 64x64 quadrant x
// K=64 = 32 MFMAs):
//   32 MFMA || {8 ds_read_b128 of a fragment half for a later phase, then one
//   half-tile of LDS-DMA (4 per lane)}  ->  lgkmcnt(0), vmcnt(24)  ->  s_barrier
// Quadrant order alternates with tile parity exactly as in v8.  Reads issued
// in phase P complete before barrier P+1, so their region is refilled in
// phase P+1; each half-tile is read 7 phases after it is issued (6 younger
// half-tiles = 24 LDS-DMA ops stay in flight across every barrier).
// Half-tile issue in tile t: ph0 W-first(t+2), ph1 W-second(t+2), ph2 XB(t+2),
// ph3 XA(t+3).  Requires an even number of K-tiles.
namespace v9 {
constexpr int BUF = 65536, WIMG = 32768;
}

template <int EPI>
__global__ __launch_bounds__(256, 1) void gemm_nt_v9(const half_t* __restrict__ A, const half_t* __restrict__ W,
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

  // staging: a half-tile = 16 pieces of 8 rows x 128 B, rows {(j>>3)*128 + (j&7)*8} (+64 for the B half);
  // wave w moves pieces 4w .. 4w+3
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ lr;
  int prow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = 4 * wave + i;
    prow[i] = (j >> 3) * 128 + (j & 7) * 8;
  }
  // per-lane 32-bit byte offsets; the K offset goes into the (scalar) base pointer so every
  // LDS-DMA is the saddr + voffset form (no per-lane 64-bit address registers)
  unsigned xo[8], wo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xo[i] = (unsigned)(min(m0 + prow[i] + lr, M - 1) * lda + lc * 8) * 2u;
    xo[4 + i] = (unsigned)(min(m0 + prow[i] + 64 + lr, M - 1) * lda + lc * 8) * 2u;
    wo[i] = (unsigned)((prow[i] + lr) * ldw + lc * 8) * 2u;
  }
  const char* Ab = (const char*)A;
  const char* Wb = (const char*)(W + (size_t)n0 * ldw);
  const size_t wb_off = (size_t)64 * ldw * 2;
#define V9_X(buf, hb, k0)                                                                         \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                \
    glds16(Ab + (size_t)(k0) * 2 + xo[(hb) * 4 + i_], smem + (buf) * v9::BUF + (prow[i_] + (hb) * 64) * 128);
#define V9_W(buf, hb, k0)                                                                         \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                \
    glds16(Wb + (hb) * wb_off + (size_t)(k0) * 2 + wo[i_], smem + (buf) * v9::BUF + v9::WIMG + (prow[i_] + (hb) * 64) * 128);

  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, grp = lane >> 4;
  const int sw = fr & 7;
  const int c0 = ((0 + grp) ^ sw) << 4;
  const int c1 = ((4 + grp) ^ sw) << 4;
  const int xrow = (wm * 128 + fr) * 128;
  const int wrow = v9::WIMG + (wn * 128 + fr) * 128;

  floatx4 acc[8][8];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  half8 xf[8][2], wf[8][2];
#define V9_FENCE_ACC()                                                                            \
  _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_)                                                \
  _Pragma("unroll") for (int t_ = 0; t_ < 8; ++t_) asm volatile("" : "+a"(acc[u_][t_]));
  // zero-init (VALU AGPR writes) must not sit right before the first asm MFMA reading them
  V9_FENCE_ACC();
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");

#define V9_RX(buf, h)                                                                             \
  _Pragma("unroll") for (int u_ = (h) * 4; u_ < (h) * 4 + 4; ++u_) {                              \
    xf[u_][0] = *(const half8*)(smem + (buf) * v9::BUF + xrow + u_ * 2048 + c0);                  \
    xf[u_][1] = *(const half8*)(smem + (buf) * v9::BUF + xrow + u_ * 2048 + c1);                  \
  }
#define V9_RW(buf, h)                                                                             \
  _Pragma("unroll") for (int t_ = (h) * 4; t_ < (h) * 4 + 4; ++t_) {                              \
    wf[t_][0] = *(const half8*)(smem + (buf) * v9::BUF + wrow + t_ * 2048 + c0);                  \
    wf[t_][1] = *(const half8*)(smem + (buf) * v9::BUF + wrow + t_ * 2048 + c1);                  \
  }
  // one phase: reads for a later phase, one half-tile of DMA, 32 MFMAs (interleaved), waits, barrier
// one phase: 32 MFMAs (k-step outer, 4x4 tiles of the quadrant) with, in issue order,
// one ds_read after each of the first 16 even-numbered MFMAs (the 8 reads of the half
// needed later) and the half-tile's 4 LDS-DMA ops after MFMAs 17, 20, 23, 26;
// then lgkmcnt(0) + counted vmcnt + barrier.  RX: 1 = read an X half, 0 = a W half.
#define V9_PHASE(xh, wh, RX, rbuf, rh, DX, dbuf, dhb, dk0)                                        \
  {                                                                                               \
    _Pragma("unroll") for (int i_ = 0; i_ < 32; ++i_) {                                           \
      const int s_ = i_ >> 4, u_ = (xh) * 4 + ((i_ >> 2) & 3), t_ = (wh) * 4 + (i_ & 3);          \
      mfma_acc_inplace_ordered(acc[u_][t_], wf[t_][s_], xf[u_][s_]);                              \
      if (i_ < 16 && (i_ & 1) == 0) {                                                             \
        const int f_ = (rh) * 4 + (i_ >> 2), k_ = (i_ >> 1) & 1;                                  \
        if (RX)                                                                                   \
          xf[f_][k_] = *(const half8*)(smem + (rbuf) * v9::BUF + xrow + f_ * 2048 + (k_ ? c1 : c0)); \
        else                                                                                      \
          wf[f_][k_] = *(const half8*)(smem + (rbuf) * v9::BUF + wrow + f_ * 2048 + (k_ ? c1 : c0)); \
      }                                                                                           \
      if (i_ >= 17 && i_ <= 26 && (i_ - 17) % 3 == 0) {                                           \
        const int p_ = (i_ - 17) / 3;                                                             \
        if (DX)                                                                                   \
          glds16(Ab + (size_t)(dk0) * 2 + xo[(dhb) * 4 + p_],                                     \
                 smem + (dbuf) * v9::BUF + (prow[p_] + (dhb) * 64) * 128);                        \
        else                                                                                      \
          glds16(Wb + (dhb) * wb_off + (size_t)(dk0) * 2 + wo[p_],                                \
                 smem + (dbuf) * v9::BUF + v9::WIMG + (prow[p_] + (dhb) * 64) * 128);             \
      }                                                                                           \
    }                                                                                             \
    __builtin_amdgcn_s_waitcnt(0xC07F);                   /* lgkmcnt(0) */                        \
    asm volatile("s_waitcnt vmcnt(24)" ::: "memory");                                             \
    __builtin_amdgcn_s_barrier();                                                                 \
  }

  const int nk = K / BK;                       // even (host-checked)
  const int kc1 = min(1, nk - 1) * BK, kc2 = min(2, nk - 1) * BK;
  // prologue: XA0 WA0 WB0 XB0 | XA1 WB1 WA1 XB1 ; read x0(0), w0(0) ; then XA2
  V9_X(0, 0, 0); V9_W(0, 0, 0); V9_W(0, 1, 0); V9_X(0, 1, 0);
  V9_X(1, 0, kc1); V9_W(1, 1, kc1); V9_W(1, 0, kc1); V9_X(1, 1, kc1);
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  V9_RX(0, 0); V9_RW(0, 0);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  V9_X(0, 0, kc2);
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  for (int kt = 0; kt < nk; kt += 2) {
    const int ka = min(kt + 2, nk - 1) * BK;   // tile kt+2 (even, buf 0)
    const int kb = min(kt + 3, nk - 1) * BK;   // tile kt+3 (odd, buf 1)
    const int kc = min(kt + 4, nk - 1) * BK;   // tile kt+4 (even, buf 0)
    // even tile kt, buf 0: W-first = WA, W-second = WB
    V9_PHASE(0, 0, 0, 0, 1, 0, 0, 0, ka);    // read w1(kt)        ; DMA WA(kt+2)
    V9_PHASE(0, 1, 1, 0, 1, 0, 0, 1, ka);    // read x1(kt)        ; DMA WB(kt+2)
    V9_PHASE(1, 1, 1, 1, 0, 1, 0, 1, ka);    // read x0(kt+1)      ; DMA XB(kt+2)
    V9_PHASE(1, 0, 0, 1, 1, 1, 1, 0, kb);    // read w1(kt+1)      ; DMA XA(kt+3)
    // odd tile kt+1, buf 1: W-first = WB, W-second = WA
    V9_PHASE(0, 1, 0, 1, 0, 0, 1, 1, kb);    // read w0(kt+1)      ; DMA WB(kt+3)
    V9_PHASE(0, 0, 1, 1, 1, 0, 1, 0, kb);    // read x1(kt+1)      ; DMA WA(kt+3)
    V9_PHASE(1, 0, 1, 0, 0, 1, 1, 1, kb);    // read x0(kt+2)      ; DMA XB(kt+3)
    V9_PHASE(1, 1, 0, 0, 0, 1, 0, 0, kc);    // read w0(kt+2)      ; DMA XA(kt+4)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // the accumulators were written by inline-asm MFMAs the hazard recognizer cannot see:
  // the nops give the last ones their passes, and the tied empty asms (ordered after the
  // nops, being volatile too) make every later AGPR read depend on them
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  V9_FENCE_ACC();
#undef V9_FENCE_ACC
#undef V9_PHASE
#undef V9_RW
#undef V9_RX
#undef V9_W
#undef V9_X

#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int m = m0 + wm * 128 + u * 16 + fr;
    if (m < M) {
#pragma unroll
      for (int p = 0; p < 4; ++p)
        store_pair<EPI>(C, ldc, m, n0 + wn * 128 + p * 32, grp, acc[u][2 * p], acc[u][2 * p + 1], ep);
    }
  }
}

// ------------------------------------------------------------------ v10
// v9 with ONE barrier per two phases (64 MFMAs): the register read-ahead stays
// one phase deep (registers are private, they need no barrier); only the
// shared-LDS hazards are synchronised, at super-phase (SP) granularity:
//   SP0 of tile t: DMA XA(t+2) + W-first(t+2)    SP1 of tile t: DMA W-second(t+2) + XB(t+2)
// (tile t's data is read in SPs 2t-1 and 2t, so each region is refilled in the
// SP after its last reads, and every half-tile is read 3 SPs after issue:
// `vmcnt(16)` = 2 SPs x 2 half-tiles x 4 ops stay in flight at each barrier).
// Original v9 notes follow.
//
// v6's geometry (4 waves = one per SIMD, 128x128 outputs per wave in 256
// AGPR accumulators: 2/3 of the LDS fragment reads per FLOP of the 8-wave
// kernels) with v8's read-ahead schedule, and the LDS reads and DMA
// interleaved INTO the MFMA stream (one wave per SIMD: nothing else would
// fill the matrix pipe while they issue).  Per phase (one 64x64 quadrant x
// K=64 = 32 MFMAs):
//   32 MFMA || {8 ds_read_b128 of a fragment half for a later phase, then one
//   half-tile of LDS-DMA (4 per lane)}  ->  lgkmcnt(0), vmcnt(24)  ->  s_barrier
// Quadrant order alternates with tile parity exactly as in v8.  Reads issued
// in phase P complete before barrier P+1, so their region is refilled in
// phase P+1; each half-tile is read 7 phases after it is issued (6 younger
// half-tiles = 24 LDS-DMA ops stay in flight across every barrier).
// Half-tile issue in tile t: ph0 W-first(t+2), ph1 W-second(t+2), ph2 XB(t+2),
// ph3 XA(t+3).  Requires an even number of K-tiles.

// ABL (ablation, main loop only): bit0 = no LDS-DMA, bit1 = no fragment ds_reads, bit2 = no waits/barriers
// SCHED: placement of a phase's 8 ds_reads / 4 LDS-DMA ops among its 32 MFMAs
//   0: reads after MFMAs 0,2,..,14; DMA after 17,20,23,26 (default)
//   1: DMA first (after 0,2,4,6), reads after 8,10,..,22
//   2: spread: reads after 0,4,..,28; DMA after 2,10,18,26
//   3: alternate from the start: read/DMA after 0..11 (r r d r r d ...), rest bare
// GM: tile order — consecutive blocks walk GM M-tiles per N-tile (grouped column-major);
// negative GM groups -GM N-tiles per M-tile instead (microbenchmark variants, 80+ in fls_gemm_ablate)
template <int EPI, int ABL = 0, int SCHED = 0, int GM = 8>
__global__ __launch_bounds__(256, 1) void gemm_nt_v10(const half_t* __restrict__ A, const half_t* __restrict__ W,
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
  int tm, tn;
  if (GM > 0) {
    constexpr int GROUP_M = GM > 0 ? GM : 1;
    const int group = bid / (GROUP_M * tiles_n);
    const int first_m = group * GROUP_M;
    const int gsz = min(tiles_m - first_m, GROUP_M);
    const int in_g = bid - group * GROUP_M * tiles_n;
    tm = first_m + in_g % gsz;
    tn = in_g / gsz;
  } else {
    constexpr int GROUP_N = GM < 0 ? -GM : 1;
    const int group = bid / (GROUP_N * tiles_m);
    const int first_n = group * GROUP_N;
    const int gsz = min(tiles_n - first_n, GROUP_N);
    const int in_g = bid - group * GROUP_N * tiles_m;
    tn = first_n + in_g % gsz;
    tm = in_g / gsz;
  }
  const int m0 = tm * BM, n0 = tn * BN;

  // staging: a half-tile = 16 pieces of 8 rows x 128 B, rows {(j>>3)*128 + (j&7)*8} (+64 for the B half);
  // wave w moves pieces 4w .. 4w+3
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ lr;
  int prow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = 4 * wave + i;
    prow[i] = (j >> 3) * 128 + (j & 7) * 8;
  }
  // per-lane 32-bit byte offsets; the K offset goes into the (scalar) base pointer so every
  // LDS-DMA is the saddr + voffset form (no per-lane 64-bit address registers)
  unsigned xo[8], wo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xo[i] = (unsigned)(min(m0 + prow[i] + lr, M - 1) * lda + lc * 8) * 2u;
    xo[4 + i] = (unsigned)(min(m0 + prow[i] + 64 + lr, M - 1) * lda + lc * 8) * 2u;
    wo[i] = (unsigned)((prow[i] + lr) * ldw + lc * 8) * 2u;
  }
  const char* Ab = (const char*)A;
  const char* Wb = (const char*)(W + (size_t)n0 * ldw);
  const size_t wb_off = (size_t)64 * ldw * 2;
#define V10_X(buf, hb, k0)                                                                         \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                \
    glds16(Ab + (size_t)(k0) * 2 + xo[(hb) * 4 + i_], smem + (buf) * v9::BUF + (prow[i_] + (hb) * 64) * 128);
#define V10_W(buf, hb, k0)                                                                         \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                \
    glds16(Wb + (hb) * wb_off + (size_t)(k0) * 2 + wo[i_], smem + (buf) * v9::BUF + v9::WIMG + (prow[i_] + (hb) * 64) * 128);

  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, grp = lane >> 4;
  const int sw = fr & 7;
  const int c0 = ((0 + grp) ^ sw) << 4;
  const int c1 = ((4 + grp) ^ sw) << 4;
  const int xrow = (wm * 128 + fr) * 128;
  const int wrow = v9::WIMG + (wn * 128 + fr) * 128;

  floatx4 acc[8][8];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  half8 xf[8][2], wf[8][2];
#define V10_FENCE_ACC()                                                                            \
  _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_)                                                \
  _Pragma("unroll") for (int t_ = 0; t_ < 8; ++t_) asm volatile("" : "+a"(acc[u_][t_]));
  // zero-init (VALU AGPR writes) must not sit right before the first asm MFMA reading them
  V10_FENCE_ACC();
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");

#define V10_RX(buf, h)                                                                             \
  _Pragma("unroll") for (int u_ = (h) * 4; u_ < (h) * 4 + 4; ++u_) {                              \
    xf[u_][0] = *(const half8*)(smem + (buf) * v9::BUF + xrow + u_ * 2048 + c0);                  \
    xf[u_][1] = *(const half8*)(smem + (buf) * v9::BUF + xrow + u_ * 2048 + c1);                  \
  }
#define V10_RW(buf, h)                                                                             \
  _Pragma("unroll") for (int t_ = (h) * 4; t_ < (h) * 4 + 4; ++t_) {                              \
    wf[t_][0] = *(const half8*)(smem + (buf) * v9::BUF + wrow + t_ * 2048 + c0);                  \
    wf[t_][1] = *(const half8*)(smem + (buf) * v9::BUF + wrow + t_ * 2048 + c1);                  \
  }
  // one phase: reads for a later phase, one half-tile of DMA, 32 MFMAs (interleaved), waits, barrier
// one phase: 32 MFMAs (k-step outer, 4x4 tiles of the quadrant) with, in issue order,
// one ds_read after each of the first 16 even-numbered MFMAs (the 8 reads of the half
// needed later) and the half-tile's 4 LDS-DMA ops after MFMAs 17, 20, 23, 26;
// then lgkmcnt(0) + counted vmcnt + barrier.  RX: 1 = read an X half, 0 = a W half.
#define V10_PHASE(xh, wh, RX, rbuf, rh, DX, dbuf, dhb, dk0, SYNC)                                        \
  {                                                                                               \
    _Pragma("unroll") for (int i_ = 0; i_ < 32; ++i_) {                                           \
      const int s_ = i_ >> 4, u_ = (xh) * 4 + ((i_ >> 2) & 3), t_ = (wh) * 4 + (i_ & 3);          \
      mfma_acc_inplace_ordered(acc[u_][t_], wf[t_][s_], xf[u_][s_]);                              \
      constexpr int rsl_[4][32] = {                                                               \
        {0,-1,1,-1,2,-1,3,-1,4,-1,5,-1,6,-1,7,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1},  \
        {-1,-1,-1,-1,-1,-1,-1,-1,0,-1,1,-1,2,-1,3,-1,4,-1,5,-1,6,-1,7,-1,-1,-1,-1,-1,-1,-1,-1,-1},  \
        {0,-1,-1,-1,1,-1,-1,-1,2,-1,-1,-1,3,-1,-1,-1,4,-1,-1,-1,5,-1,-1,-1,6,-1,-1,-1,7,-1,-1,-1},  \
        {0,1,-1,2,3,-1,4,5,-1,6,7,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1}}; \
      constexpr int dsl_[4][32] = {                                                               \
        {-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,0,-1,-1,1,-1,-1,2,-1,-1,3,-1,-1,-1,-1,-1},\
        {0,-1,1,-1,2,-1,3,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1},\
        {-1,-1,0,-1,-1,-1,-1,-1,-1,-1,1,-1,-1,-1,-1,-1,-1,-1,2,-1,-1,-1,-1,-1,-1,-1,3,-1,-1,-1,-1,-1},\
        {-1,-1,0,-1,-1,1,-1,-1,2,-1,-1,3,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1,-1}};\
      const int rj_ = rsl_[SCHED][i_], dj_ = dsl_[SCHED][i_];                                     \
      if (!(ABL & 2) && rj_ >= 0) {                                                               \
        const int f_ = (rh) * 4 + (rj_ >> 1), k_ = rj_ & 1;                                       \
        if (RX)                                                                                   \
          xf[f_][k_] = *(const half8*)(smem + (rbuf) * v9::BUF + xrow + f_ * 2048 + (k_ ? c1 : c0)); \
        else                                                                                      \
          wf[f_][k_] = *(const half8*)(smem + (rbuf) * v9::BUF + wrow + f_ * 2048 + (k_ ? c1 : c0)); \
      }                                                                                           \
      if (!(ABL & 1) && dj_ >= 0) {                                                               \
        const int p_ = dj_;                                                                       \
        if (DX)                                                                                   \
          glds16(Ab + (size_t)(dk0) * 2 + xo[(dhb) * 4 + p_],                                     \
                 smem + (dbuf) * v9::BUF + (prow[p_] + (dhb) * 64) * 128);                        \
        else                                                                                      \
          glds16(Wb + (dhb) * wb_off + (size_t)(dk0) * 2 + wo[p_],                                \
                 smem + (dbuf) * v9::BUF + v9::WIMG + (prow[p_] + (dhb) * 64) * 128);             \
      }                                                                                           \
    }                                                                                             \
    if (SYNC && !(ABL & 4)) {                                                                     \
      __builtin_amdgcn_s_waitcnt(0xC07F);                 /* lgkmcnt(0) */                        \
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");                                           \
      __builtin_amdgcn_s_barrier();                                                               \
    }                                                                                             \
  }

  const int nk = K / BK;                       // even (host-checked)
  const int kc1 = min(1, nk - 1) * BK;
  // prologue = virtual SPs -4..-1: [XA0 WA0] [WB0 XB0] [XA1 WB1] [WA1 XB1]
  V10_X(0, 0, 0); V10_W(0, 0, 0); V10_W(0, 1, 0); V10_X(0, 1, 0);
  V10_X(1, 0, kc1); V10_W(1, 1, kc1); V10_W(1, 0, kc1); V10_X(1, 1, kc1);
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  V10_RX(0, 0); V10_RW(0, 0);                  // SP -1's reads: x0(0), w0(0)
  __builtin_amdgcn_s_waitcnt(0xC07F);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; kt += 2) {
    const int ka = min(kt + 2, nk - 1) * BK;   // tile kt+2 -> buf 0
    const int kb = min(kt + 3, nk - 1) * BK;   // tile kt+3 -> buf 1
    // even tile kt (buf 0; W-first = WA, W-second = WB)
    V10_PHASE(0, 0, 0, 0, 1, 1, 0, 0, ka, 0);  // read w1(kt)   ; DMA XA(kt+2)
    V10_PHASE(0, 1, 1, 0, 1, 0, 0, 0, ka, 1);  // read x1(kt)   ; DMA WA(kt+2)   | sync
    V10_PHASE(1, 1, 1, 1, 0, 0, 0, 1, ka, 0);  // read x0(kt+1) ; DMA WB(kt+2)
    V10_PHASE(1, 0, 0, 1, 1, 1, 0, 1, ka, 1);  // read w1(kt+1) ; DMA XB(kt+2)   | sync
    // odd tile kt+1 (buf 1; W-first = WB, W-second = WA)
    V10_PHASE(0, 1, 0, 1, 0, 1, 1, 0, kb, 0);  // read w0(kt+1) ; DMA XA(kt+3)
    V10_PHASE(0, 0, 1, 1, 1, 0, 1, 1, kb, 1);  // read x1(kt+1) ; DMA WB(kt+3)   | sync
    V10_PHASE(1, 0, 1, 0, 0, 0, 1, 0, kb, 0);  // read x0(kt+2) ; DMA WA(kt+3)
    V10_PHASE(1, 1, 0, 0, 0, 1, 1, 1, kb, 1);  // read w0(kt+2) ; DMA XB(kt+3)   | sync
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // the accumulators were written by inline-asm MFMAs the hazard recognizer cannot see:
  // the nops give the last ones their passes, and the tied empty asms (ordered after the
  // nops, being volatile too) make every later AGPR read depend on them
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  V10_FENCE_ACC();
#undef V10_FENCE_ACC
#undef V10_PHASE
#undef V10_RW
#undef V10_RX
#undef V10_W
#undef V10_X

  epilogue_quadrant<EPI>(C, ldc, M, m0 + wm * 128 + fr, n0 + wn * 128, grp, acc, ep);
}

// ------------------------------------------------------------------ v13
// Persistent v10: the grid is one block per CU (multiple of 8, so virtual tile id
// v = blockIdx.x + i * gridDim.x stays on the XCD that v10's remap assumes) and each
// block walks its tiles in the same remapped / grouped order as v10.  With one
// block per CU (256 AGPR accumulators, 128 KiB LDS) v10 leaves the CU idle while a
// tile's epilogue stores drain and while the next block's first K-tiles are in flight
// (the fixed per-tile cost of the K sweep, profiles/r1_gemm_study/k_sweep.log:
// 3-5% of the 70B projections).  Here the next tile's 2-stage prologue DMA is issued
// BEFORE the current tile's epilogue, so the HBM/L2 latency of the first K-tiles
// overlaps the epilogue's loads and stores.  Main loop identical to v10 (SCHED 0).
template <int EPI, int GM = 8>
__global__ __launch_bounds__(256, 1) void gemm_nt_v13(const half_t* __restrict__ A, const half_t* __restrict__ W,
                                                    half_t* __restrict__ C, int M, int N, int K, int lda, int ldw,
                                                    int ldc, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int tiles_m = (M + BM - 1) / BM;
  const int tiles_n = N / BN;
  const int ntiles = tiles_m * tiles_n;
  const int q8 = ntiles >> 3, r8 = ntiles & 7;
  int m0, n0;
#define V13_TILE(v)                                                                                 \
  {                                                                                                 \
    const int xcd_ = (v) & 7, loc_ = (v) >> 3;                                                      \
    const int b_ = (xcd_ < r8 ? xcd_ * (q8 + 1) : r8 * (q8 + 1) + (xcd_ - r8) * q8) + loc_;         \
    int tm_, tn_;                                                                                   \
    if (GM > 0) {                                                                                   \
      constexpr int GROUP_M = GM > 0 ? GM : 1;                                                      \
      const int group_ = b_ / (GROUP_M * tiles_n);                                                  \
      const int first_ = group_ * GROUP_M;                                                          \
      const int gsz_ = min(tiles_m - first_, GROUP_M);                                              \
      const int in_ = b_ - group_ * GROUP_M * tiles_n;                                              \
      tm_ = first_ + in_ % gsz_;                                                                    \
      tn_ = in_ / gsz_;                                                                             \
    } else {                                                                                        \
      constexpr int GROUP_N = GM < 0 ? -GM : 1;                                                     \
      const int group_ = b_ / (GROUP_N * tiles_m);                                                  \
      const int first_ = group_ * GROUP_N;                                                          \
      const int gsz_ = min(tiles_n - first_, GROUP_N);                                              \
      const int in_ = b_ - group_ * GROUP_N * tiles_m;                                              \
      tn_ = first_ + in_ % gsz_;                                                                    \
      tm_ = in_ / gsz_;                                                                             \
    }                                                                                               \
    m0 = tm_ * BM;                                                                                  \
    n0 = tn_ * BN;                                                                                  \
  }

  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ lr;
  int prow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = 4 * wave + i;
    prow[i] = (j >> 3) * 128 + (j & 7) * 8;
  }
  unsigned xo[8], wo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) wo[i] = (unsigned)((prow[i] + lr) * ldw + lc * 8) * 2u;
  const char* Ab = (const char*)A;
  const char* Wb;
  const size_t wb_off = (size_t)64 * ldw * 2;
#define V13_SETUP()                                                                                 \
  {                                                                                                 \
    _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_) {                                              \
      xo[i_] = (unsigned)(min(m0 + prow[i_] + lr, M - 1) * lda + lc * 8) * 2u;                      \
      xo[4 + i_] = (unsigned)(min(m0 + prow[i_] + 64 + lr, M - 1) * lda + lc * 8) * 2u;             \
    }                                                                                               \
    Wb = (const char*)(W + (size_t)n0 * ldw);                                                       \
  }
#define V13_X(buf, hb, k0)                                                                         \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                \
    glds16(Ab + (size_t)(k0) * 2 + xo[(hb) * 4 + i_], smem + (buf) * v9::BUF + (prow[i_] + (hb) * 64) * 128);
#define V13_W(buf, hb, k0)                                                                         \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                \
    glds16(Wb + (hb) * wb_off + (size_t)(k0) * 2 + wo[i_], smem + (buf) * v9::BUF + v9::WIMG + (prow[i_] + (hb) * 64) * 128);

  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, grp = lane >> 4;
  const int sw = fr & 7;
  const int c0 = ((0 + grp) ^ sw) << 4;
  const int c1 = ((4 + grp) ^ sw) << 4;
  const int xrow = (wm * 128 + fr) * 128;
  const int wrow = v9::WIMG + (wn * 128 + fr) * 128;

  floatx4 acc[8][8];
  half8 xf[8][2], wf[8][2];
#define V13_FENCE_ACC()                                                                            \
  _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_)                                                \
  _Pragma("unroll") for (int t_ = 0; t_ < 8; ++t_) asm volatile("" : "+a"(acc[u_][t_]));
#define V13_RX(buf, h)                                                                             \
  _Pragma("unroll") for (int u_ = (h) * 4; u_ < (h) * 4 + 4; ++u_) {                              \
    xf[u_][0] = *(const half8*)(smem + (buf) * v9::BUF + xrow + u_ * 2048 + c0);                  \
    xf[u_][1] = *(const half8*)(smem + (buf) * v9::BUF + xrow + u_ * 2048 + c1);                  \
  }
#define V13_RW(buf, h)                                                                             \
  _Pragma("unroll") for (int t_ = (h) * 4; t_ < (h) * 4 + 4; ++t_) {                              \
    wf[t_][0] = *(const half8*)(smem + (buf) * v9::BUF + wrow + t_ * 2048 + c0);                  \
    wf[t_][1] = *(const half8*)(smem + (buf) * v9::BUF + wrow + t_ * 2048 + c1);                  \
  }
// v10's phase with SCHED 0 (reads after even MFMAs 0..14, DMA after MFMAs 17, 20, 23, 26)
#define V13_PHASE(xh, wh, RX, rbuf, rh, DX, dbuf, dhb, dk0, SYNC)                                  \
  {                                                                                               \
    _Pragma("unroll") for (int i_ = 0; i_ < 32; ++i_) {                                           \
      const int s_ = i_ >> 4, u_ = (xh) * 4 + ((i_ >> 2) & 3), t_ = (wh) * 4 + (i_ & 3);          \
      mfma_acc_inplace_ordered(acc[u_][t_], wf[t_][s_], xf[u_][s_]);                              \
      if (i_ < 16 && (i_ & 1) == 0) {                                                             \
        const int rj_ = i_ >> 1;                                                                  \
        const int f_ = (rh) * 4 + (rj_ >> 1), k_ = rj_ & 1;                                       \
        if (RX)                                                                                   \
          xf[f_][k_] = *(const half8*)(smem + (rbuf) * v9::BUF + xrow + f_ * 2048 + (k_ ? c1 : c0)); \
        else                                                                                      \
          wf[f_][k_] = *(const half8*)(smem + (rbuf) * v9::BUF + wrow + f_ * 2048 + (k_ ? c1 : c0)); \
      }                                                                                           \
      if (i_ >= 17 && i_ <= 26 && (i_ - 17) % 3 == 0) {                                           \
        const int p_ = (i_ - 17) / 3;                                                             \
        if (DX)                                                                                   \
          glds16(Ab + (size_t)(dk0) * 2 + xo[(dhb) * 4 + p_],                                     \
                 smem + (dbuf) * v9::BUF + (prow[p_] + (dhb) * 64) * 128);                        \
        else                                                                                      \
          glds16(Wb + (dhb) * wb_off + (size_t)(dk0) * 2 + wo[p_],                                \
                 smem + (dbuf) * v9::BUF + v9::WIMG + (prow[p_] + (dhb) * 64) * 128);             \
      }                                                                                           \
    }                                                                                             \
    if (SYNC) {                                                                                   \
      __builtin_amdgcn_s_waitcnt(0xC07F);                 /* lgkmcnt(0) */                        \
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");                                           \
      __builtin_amdgcn_s_barrier();                                                               \
    }                                                                                             \
  }

  const int nk = K / BK;                       // even (host-checked)
  const int kc1 = min(1, nk - 1) * BK;
#define V13_PROLOGUE_DMA()                                                                         \
  V13_X(0, 0, 0); V13_W(0, 0, 0); V13_W(0, 1, 0); V13_X(0, 1, 0);                                 \
  V13_X(1, 0, kc1); V13_W(1, 1, kc1); V13_W(1, 0, kc1); V13_X(1, 1, kc1);

  int v = blockIdx.x;
  V13_TILE(v);
  V13_SETUP();
  V13_PROLOGUE_DMA();
  bool first = true;
  while (true) {
    if (first) {
      asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    } else {
      // the prologue DMA was issued before the previous tile's epilogue loads / stores:
      // vmcnt cannot count it apart from them
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    V13_FENCE_ACC();
    V13_RX(0, 0); V13_RW(0, 0);                // SP -1's reads: x0(0), w0(0)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // zero-init (VALU AGPR writes) must not sit right before the first asm MFMA reading them
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    for (int kt = 0; kt < nk; kt += 2) {
      const int ka = min(kt + 2, nk - 1) * BK;
      const int kb = min(kt + 3, nk - 1) * BK;
      V13_PHASE(0, 0, 0, 0, 1, 1, 0, 0, ka, 0);
      V13_PHASE(0, 1, 1, 0, 1, 0, 0, 0, ka, 1);
      V13_PHASE(1, 1, 1, 1, 0, 0, 0, 1, ka, 0);
      V13_PHASE(1, 0, 0, 1, 1, 1, 0, 1, ka, 1);
      V13_PHASE(0, 1, 0, 1, 0, 1, 1, 0, kb, 0);
      V13_PHASE(0, 0, 1, 1, 1, 0, 1, 1, kb, 1);
      V13_PHASE(1, 0, 1, 0, 0, 0, 1, 0, kb, 0);
      V13_PHASE(1, 1, 0, 0, 0, 1, 1, 1, kb, 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    V13_FENCE_ACC();
    const int em0 = m0, en0 = n0;
    v += gridDim.x;
    const bool more = v < ntiles;              // block-uniform
    if (more) {
      // every wave's LDS reads (lgkmcnt(0) before the last phase's barrier) and DMA
      // (vmcnt(0) above) of this tile are complete once all waves pass this barrier
      __builtin_amdgcn_s_barrier();
      V13_TILE(v);
      V13_SETUP();
      V13_PROLOGUE_DMA();
    }
    epilogue_quadrant<EPI>(C, ldc, M, em0 + wm * 128 + fr, en0 + wn * 128, grp, acc, ep);
    if (!more) break;
    first = false;
  }
#undef V13_PROLOGUE_DMA
#undef V13_FENCE_ACC
#undef V13_PHASE
#undef V13_RW
#undef V13_RX
#undef V13_W
#undef V13_X
#undef V13_SETUP
#undef V13_TILE
}

// ------------------------------------------------------------------ v11
// v10 with the LDS-DMA issued as `buffer_load_dwordx4 ... offen lds` from a
// buffer resource: every piece of an operand uses the SAME per-lane VGPR
// offset (row-in-piece x ld + swizzled chunk) and a wave-uniform SGPR offset
// (piece row base x ld + k), so the DMA costs no per-piece vector address
// registers or VALU; rows past M read as zero (buffer range check) instead of
// being clamped.  Schedule identical to v10.

// v9 with ONE barrier per two phases (64 MFMAs): the register read-ahead stays
// one phase deep (registers are private, they need no barrier); only the
// shared-LDS hazards are synchronised, at super-phase (SP) granularity:
//   SP0 of tile t: DMA XA(t+2) + W-first(t+2)    SP1 of tile t: DMA W-second(t+2) + XB(t+2)
// (tile t's data is read in SPs 2t-1 and 2t, so each region is refilled in the
// SP after its last reads, and every half-tile is read 3 SPs after issue:
// `vmcnt(16)` = 2 SPs x 2 half-tiles x 4 ops stay in flight at each barrier).
// Original v9 notes follow.
//
// v6's geometry (4 waves = one per SIMD, 128x128 outputs per wave in 256
// AGPR accumulators: 2/3 of the LDS fragment reads per FLOP of the 8-wave
// kernels) with v8's read-ahead schedule, and the LDS reads and DMA
// interleaved INTO the MFMA stream (one wave per SIMD: nothing else would
// fill the matrix pipe while they issue).  Per phase (one 64x64 quadrant x
// K=64 = 32 MFMAs):
//   32 MFMA || {8 ds_read_b128 of a fragment half for a later phase, then one
//   half-tile of LDS-DMA (4 per lane)}  ->  lgkmcnt(0), vmcnt(24)  ->  s_barrier
// Quadrant order alternates with tile parity exactly as in v8.  Reads issued
// in phase P complete before barrier P+1, so their region is refilled in
// phase P+1; each half-tile is read 7 phases after it is issued (6 younger
// half-tiles = 24 LDS-DMA ops stay in flight across every barrier).
// Half-tile issue in tile t: ph0 W-first(t+2), ph1 W-second(t+2), ph2 XB(t+2),
// ph3 XA(t+3).  Requires an even number of K-tiles.

// ABL (ablation, main loop only): bit0 = no LDS-DMA, bit1 = no fragment ds_reads, bit2 = no waits/barriers
template <int EPI, int ABL = 0>
__global__ __launch_bounds__(256, 1) void gemm_nt_v11(const half_t* __restrict__ A, const half_t* __restrict__ W,
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

  // staging: a half-tile = 16 pieces of 8 rows x 128 B, rows {(j>>3)*128 + (j&7)*8} (+64 for the B half);
  // wave w moves pieces 4w .. 4w+3
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ lr;
  int prow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = 4 * wave + i;
    prow[i] = (j >> 3) * 128 + (j & 7) * 8;
  }
  // buffer resources: X = whole matrix (rows >= M fall outside num_records -> 0), W = this block's 256 rows
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, M * lda * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (size_t)n0 * ldw), (short)0,
                                                                       BN * ldw * 2, 0x00020000);
  const unsigned xv = (unsigned)(lr * lda + lc * 8) * 2u;      // per-lane, shared by every X piece
  const unsigned wv = (unsigned)(lr * ldw + lc * 8) * 2u;      // per-lane, shared by every W piece
  unsigned xs[4], ws[4];                                       // wave-uniform piece bases (bytes)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xs[i] = (unsigned)((m0 + prow[i]) * lda) * 2u;
    ws[i] = (unsigned)(prow[i] * ldw) * 2u;
  }
  const unsigned xhb = (unsigned)(64 * lda) * 2u, whb = (unsigned)(64 * ldw) * 2u;
#define V11_BLD(rsrc, lds, voff, soff)                                                            \
  __builtin_amdgcn_raw_ptr_buffer_load_lds((rsrc), (LDS_AS void*)(lds), 16, (voff), (soff), 0, 0)
#define V11_X(buf, hb, k0)                                                                        \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                \
    V11_BLD(xr, smem + (buf) * v9::BUF + (prow[i_] + (hb) * 64) * 128, xv,                        \
            xs[i_] + (hb) * xhb + (unsigned)(k0) * 2u);
#define V11_W(buf, hb, k0)                                                                        \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                \
    V11_BLD(wr, smem + (buf) * v9::BUF + v9::WIMG + (prow[i_] + (hb) * 64) * 128, wv,             \
            ws[i_] + (hb) * whb + (unsigned)(k0) * 2u);

  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, grp = lane >> 4;
  const int sw = fr & 7;
  const int c0 = ((0 + grp) ^ sw) << 4;
  const int c1 = ((4 + grp) ^ sw) << 4;
  const int xrow = (wm * 128 + fr) * 128;
  const int wrow = v9::WIMG + (wn * 128 + fr) * 128;

  floatx4 acc[8][8];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  half8 xf[8][2], wf[8][2];
#define V11_FENCE_ACC()                                                                            \
  _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_)                                                \
  _Pragma("unroll") for (int t_ = 0; t_ < 8; ++t_) asm volatile("" : "+a"(acc[u_][t_]));
  // zero-init (VALU AGPR writes) must not sit right before the first asm MFMA reading them
  V11_FENCE_ACC();
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");

#define V11_RX(buf, h)                                                                             \
  _Pragma("unroll") for (int u_ = (h) * 4; u_ < (h) * 4 + 4; ++u_) {                              \
    xf[u_][0] = *(const half8*)(smem + (buf) * v9::BUF + xrow + u_ * 2048 + c0);                  \
    xf[u_][1] = *(const half8*)(smem + (buf) * v9::BUF + xrow + u_ * 2048 + c1);                  \
  }
#define V11_RW(buf, h)                                                                             \
  _Pragma("unroll") for (int t_ = (h) * 4; t_ < (h) * 4 + 4; ++t_) {                              \
    wf[t_][0] = *(const half8*)(smem + (buf) * v9::BUF + wrow + t_ * 2048 + c0);                  \
    wf[t_][1] = *(const half8*)(smem + (buf) * v9::BUF + wrow + t_ * 2048 + c1);                  \
  }
  // one phase: reads for a later phase, one half-tile of DMA, 32 MFMAs (interleaved), waits, barrier
// one phase: 32 MFMAs (k-step outer, 4x4 tiles of the quadrant) with, in issue order,
// one ds_read after each of the first 16 even-numbered MFMAs (the 8 reads of the half
// needed later) and the half-tile's 4 LDS-DMA ops after MFMAs 17, 20, 23, 26;
// then lgkmcnt(0) + counted vmcnt + barrier.  RX: 1 = read an X half, 0 = a W half.
#define V11_PHASE(xh, wh, RX, rbuf, rh, DX, dbuf, dhb, dk0, SYNC)                                        \
  {                                                                                               \
    _Pragma("unroll") for (int i_ = 0; i_ < 32; ++i_) {                                           \
      const int s_ = i_ >> 4, u_ = (xh) * 4 + ((i_ >> 2) & 3), t_ = (wh) * 4 + (i_ & 3);          \
      mfma_acc_inplace_ordered(acc[u_][t_], wf[t_][s_], xf[u_][s_]);                              \
      if (!(ABL & 2) && i_ < 16 && (i_ & 1) == 0) {                                               \
        const int f_ = (rh) * 4 + (i_ >> 2), k_ = (i_ >> 1) & 1;                                  \
        if (RX)                                                                                   \
          xf[f_][k_] = *(const half8*)(smem + (rbuf) * v9::BUF + xrow + f_ * 2048 + (k_ ? c1 : c0)); \
        else                                                                                      \
          wf[f_][k_] = *(const half8*)(smem + (rbuf) * v9::BUF + wrow + f_ * 2048 + (k_ ? c1 : c0)); \
      }                                                                                           \
      if (!(ABL & 1) && i_ >= 17 && i_ <= 26 && (i_ - 17) % 3 == 0) {                             \
        const int p_ = (i_ - 17) / 3;                                                             \
        if (DX)                                                                                   \
          V11_BLD(xr, smem + (dbuf) * v9::BUF + (prow[p_] + (dhb) * 64) * 128, xv,                \
                  xs[p_] + (dhb) * xhb + (unsigned)(dk0) * 2u);                                   \
        else                                                                                      \
          V11_BLD(wr, smem + (dbuf) * v9::BUF + v9::WIMG + (prow[p_] + (dhb) * 64) * 128, wv,     \
                  ws[p_] + (dhb) * whb + (unsigned)(dk0) * 2u);                                   \
      }                                                                                           \
    }                                                                                             \
    if (SYNC && !(ABL & 4)) {                                                                     \
      __builtin_amdgcn_s_waitcnt(0xC07F);                 /* lgkmcnt(0) */                        \
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");                                           \
      __builtin_amdgcn_s_barrier();                                                               \
    }                                                                                             \
  }

  const int nk = K / BK;                       // even (host-checked)
  const int kc1 = min(1, nk - 1) * BK;
  // prologue = virtual SPs -4..-1: [XA0 WA0] [WB0 XB0] [XA1 WB1] [WA1 XB1]
  V11_X(0, 0, 0); V11_W(0, 0, 0); V11_W(0, 1, 0); V11_X(0, 1, 0);
  V11_X(1, 0, kc1); V11_W(1, 1, kc1); V11_W(1, 0, kc1); V11_X(1, 1, kc1);
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  V11_RX(0, 0); V11_RW(0, 0);                  // SP -1's reads: x0(0), w0(0)
  __builtin_amdgcn_s_waitcnt(0xC07F);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; kt += 2) {
    const int ka = min(kt + 2, nk - 1) * BK;   // tile kt+2 -> buf 0
    const int kb = min(kt + 3, nk - 1) * BK;   // tile kt+3 -> buf 1
    // even tile kt (buf 0; W-first = WA, W-second = WB)
    V11_PHASE(0, 0, 0, 0, 1, 1, 0, 0, ka, 0);  // read w1(kt)   ; DMA XA(kt+2)
    V11_PHASE(0, 1, 1, 0, 1, 0, 0, 0, ka, 1);  // read x1(kt)   ; DMA WA(kt+2)   | sync
    V11_PHASE(1, 1, 1, 1, 0, 0, 0, 1, ka, 0);  // read x0(kt+1) ; DMA WB(kt+2)
    V11_PHASE(1, 0, 0, 1, 1, 1, 0, 1, ka, 1);  // read w1(kt+1) ; DMA XB(kt+2)   | sync
    // odd tile kt+1 (buf 1; W-first = WB, W-second = WA)
    V11_PHASE(0, 1, 0, 1, 0, 1, 1, 0, kb, 0);  // read w0(kt+1) ; DMA XA(kt+3)
    V11_PHASE(0, 0, 1, 1, 1, 0, 1, 1, kb, 1);  // read x1(kt+1) ; DMA WB(kt+3)   | sync
    V11_PHASE(1, 0, 1, 0, 0, 0, 1, 0, kb, 0);  // read x0(kt+2) ; DMA WA(kt+3)
    V11_PHASE(1, 1, 0, 0, 0, 1, 1, 1, kb, 1);  // read w0(kt+2) ; DMA XB(kt+3)   | sync
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // the accumulators were written by inline-asm MFMAs the hazard recognizer cannot see:
  // the nops give the last ones their passes, and the tied empty asms (ordered after the
  // nops, being volatile too) make every later AGPR read depend on them
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  V11_FENCE_ACC();
#undef V11_FENCE_ACC
#undef V11_PHASE
#undef V11_RW
#undef V11_RX
#undef V11_W
#undef V11_X
#undef V11_BLD

#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int m = m0 + wm * 128 + u * 16 + fr;
    if (m < M) {
#pragma unroll
      for (int p = 0; p < 4; ++p)
        store_pair<EPI>(C, ldc, m, n0 + wn * 128 + p * 32, grp, acc[u][2 * p], acc[u][2 * p + 1], ep);
    }
  }
}

// ------------------------------------------------------------------ v12
// v10's schedule on v_mfma_f32_32x32x16_f16: the wave's 128x128 quadrant is
// 4 x 4 blocks of 32x32 (16 floatx16 = 256 AGPRs), a phase = one 64x64 quadrant
// x K=64 = 16 MFMAs (same matrix-pipe time as v10's 32 16x16x32 ones, half the
// instructions).  A fragment half = 2 blocks x 4 k-steps = 8 half8, read one
// phase ahead exactly as in v10; the 32x32 layout puts a lane's 4-row groups
// 8 apart, so RoPE / SwiGLU partners (16 apart) are element groups g, g+2 of
// the same lane.
template <int EPI, int ABL = 0>
__global__ __launch_bounds__(256, 1) void gemm_nt_v12(const half_t* __restrict__ A, const half_t* __restrict__ W,
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

  // staging: identical to v10 (half-tiles XA/XB = X rows {0-63,128-191}/{64-127,192-255}, WA/WB likewise)
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ lr;
  int prow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = 4 * wave + i;
    prow[i] = (j >> 3) * 128 + (j & 7) * 8;
  }
  unsigned xo[8], wo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xo[i] = (unsigned)(min(m0 + prow[i] + lr, M - 1) * lda + lc * 8) * 2u;
    xo[4 + i] = (unsigned)(min(m0 + prow[i] + 64 + lr, M - 1) * lda + lc * 8) * 2u;
    wo[i] = (unsigned)((prow[i] + lr) * ldw + lc * 8) * 2u;
  }
  const char* Ab = (const char*)A;
  const char* Wb = (const char*)(W + (size_t)n0 * ldw);
  const size_t wb_off = (size_t)64 * ldw * 2;
#define V12_X(buf, hb, k0)                                                                        \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                \
    glds16(Ab + (size_t)(k0) * 2 + xo[(hb) * 4 + i_], smem + (buf) * v9::BUF + (prow[i_] + (hb) * 64) * 128);
#define V12_W(buf, hb, k0)                                                                        \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                \
    glds16(Wb + (hb) * wb_off + (size_t)(k0) * 2 + wo[i_],                                        \
           smem + (buf) * v9::BUF + v9::WIMG + (prow[i_] + (hb) * 64) * 128);

  // fragments: lane reads row (lane & 31) of a 32-row block, 16-B chunk 2s + (lane >> 5)
  const int wm = wave >> 1, wn = wave & 1;
  const int r32 = lane & 31, hi = lane >> 5, sw = lane & 7;
  const int xrow = (wm * 128 + r32) * 128;
  const int wrow = v9::WIMG + (wn * 128 + r32) * 128;
  int ch[4];
#pragma unroll
  for (int st = 0; st < 4; ++st) ch[st] = ((2 * st + hi) ^ sw) << 4;

  floatx16 acc[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[u][t][e] = 0.f;
  half8 xf[4][4], wf[4][4];           // [32-row block][k-step]
#define V12_FENCE_ACC()                                                                           \
  _Pragma("unroll") for (int u_ = 0; u_ < 4; ++u_)                                                \
  _Pragma("unroll") for (int t_ = 0; t_ < 4; ++t_) asm volatile("" : "+a"(acc[u_][t_]));
  V12_FENCE_ACC();
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");

#define V12_RX(buf, h)                                                                            \
  _Pragma("unroll") for (int j_ = 0; j_ < 8; ++j_)                                                \
    xf[(h) * 2 + (j_ >> 2)][j_ & 3] =                                                             \
        *(const half8*)(smem + (buf) * v9::BUF + xrow + ((h) * 2 + (j_ >> 2)) * 4096 + ch[j_ & 3]);
#define V12_RW(buf, h)                                                                            \
  _Pragma("unroll") for (int j_ = 0; j_ < 8; ++j_)                                                \
    wf[(h) * 2 + (j_ >> 2)][j_ & 3] =                                                             \
        *(const half8*)(smem + (buf) * v9::BUF + wrow + ((h) * 2 + (j_ >> 2)) * 4096 + ch[j_ & 3]);
  // phase: 16 MFMAs (k-step outer); one read after each of MFMAs 0..7; DMA after 8, 10, 12, 14
#define V12_PHASE(xh, wh, RX, rbuf, rh, DX, dbuf, dhb, dk0, SYNC)                                  \
  {                                                                                               \
    _Pragma("unroll") for (int i_ = 0; i_ < 16; ++i_) {                                           \
      const int s_ = i_ >> 2, u_ = (xh) * 2 + ((i_ >> 1) & 1), t_ = (wh) * 2 + (i_ & 1);          \
      mfma32_acc_inplace_ordered(acc[u_][t_], wf[t_][s_], xf[u_][s_]);                            \
      if (!(ABL & 2) && i_ < 8) {                                                                 \
        const int b_ = (rh) * 2 + (i_ >> 2), k_ = i_ & 3;                                         \
        if (RX)                                                                                   \
          xf[b_][k_] = *(const half8*)(smem + (rbuf) * v9::BUF + xrow + b_ * 4096 + ch[k_]);      \
        else                                                                                      \
          wf[b_][k_] = *(const half8*)(smem + (rbuf) * v9::BUF + wrow + b_ * 4096 + ch[k_]);      \
      }                                                                                           \
      if (!(ABL & 1) && i_ >= 8 && (i_ & 1) == 0) {                                               \
        const int p_ = (i_ - 8) >> 1;                                                             \
        if (DX)                                                                                   \
          glds16(Ab + (size_t)(dk0) * 2 + xo[(dhb) * 4 + p_],                                     \
                 smem + (dbuf) * v9::BUF + (prow[p_] + (dhb) * 64) * 128);                        \
        else                                                                                      \
          glds16(Wb + (dhb) * wb_off + (size_t)(dk0) * 2 + wo[p_],                                \
                 smem + (dbuf) * v9::BUF + v9::WIMG + (prow[p_] + (dhb) * 64) * 128);             \
      }                                                                                           \
    }                                                                                             \
    if (SYNC) {                                                                                   \
      __builtin_amdgcn_s_waitcnt(0xC07F);                                                         \
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");                                           \
      __builtin_amdgcn_s_barrier();                                                               \
    }                                                                                             \
  }

  const int nk = K / BK;
  const int kc1 = min(1, nk - 1) * BK;
  V12_X(0, 0, 0); V12_W(0, 0, 0); V12_W(0, 1, 0); V12_X(0, 1, 0);
  V12_X(1, 0, kc1); V12_W(1, 1, kc1); V12_W(1, 0, kc1); V12_X(1, 1, kc1);
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  V12_RX(0, 0); V12_RW(0, 0);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; kt += 2) {
    const int ka = min(kt + 2, nk - 1) * BK;
    const int kb = min(kt + 3, nk - 1) * BK;
    V12_PHASE(0, 0, 0, 0, 1, 1, 0, 0, ka, 0);
    V12_PHASE(0, 1, 1, 0, 1, 0, 0, 0, ka, 1);
    V12_PHASE(1, 1, 1, 1, 0, 0, 0, 1, ka, 0);
    V12_PHASE(1, 0, 0, 1, 1, 1, 0, 1, ka, 1);
    V12_PHASE(0, 1, 0, 1, 0, 1, 1, 0, kb, 0);
    V12_PHASE(0, 0, 1, 1, 1, 0, 1, 1, kb, 1);
    V12_PHASE(1, 0, 1, 0, 0, 0, 1, 0, kb, 0);
    V12_PHASE(1, 1, 0, 0, 0, 1, 1, 1, kb, 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  V12_FENCE_ACC();
#undef V12_FENCE_ACC
#undef V12_PHASE
#undef V12_RW
#undef V12_RX
#undef V12_W
#undef V12_X

#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int m = m0 + wm * 128 + u * 32 + r32;
    if (m < M) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int nb = n0 + wn * 128 + t * 32;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          const floatx4 a = {acc[u][t][4 * g], acc[u][t][4 * g + 1], acc[u][t][4 * g + 2], acc[u][t][4 * g + 3]};
          const floatx4 c = {acc[u][t][4 * g + 8], acc[u][t][4 * g + 9], acc[u][t][4 * g + 10],
                             acc[u][t][4 * g + 11]};
          store_pair_off<EPI>(C, ldc, m, nb, 8 * g + 4 * hi, a, c, ep);
        }
      }
    }
  }
}

int g_variant = -1;   // -1: from env FLS_GEMM_VARIANT (default 3)
int g_v10_order = 0;  // 0: by shape (launch<EPI>), else a fixed GM (fls_gemm_set_order)
int g_rope_persistent = 1;  // variant 10: QKV + RoPE GEMMs on the persistent v13 (fls_gemm_set_rope_persistent)

int variant() {
  if (g_variant < 0) {
    const char* e = getenv("FLS_GEMM_VARIANT");
    g_variant = e ? atoi(e) : 10;
  }
  return g_variant;
}

int g_mid = -1;   // mid-M kernel: -1 = from FLS_GEMM_MID (default on), 0 = off, 1 = on

bool mid_enabled() {
  if (g_mid < 0) {
    const char* e = getenv("FLS_GEMM_MID");
    g_mid = e ? (atoi(e) != 0) : 1;
  }
  return g_mid != 0;
}

template <int EPI>
int launch(const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda, int ldw, int ldc,
           const Epi& ep, hipStream_t s) {
  // Too few 256x256 tiles for 256 CUs -> 64x128 tiles.  Measured crossover
  // (profiles/r1_gemm_mid): the mid kernel wins below ~128 main tiles, and at
  // M <= 64 (3/4 of every 256-row tile wasted) up to 512; above that its lower
  // L2 reuse (43 vs 128 FLOP per staged byte) costs more than the idle CUs.
  const size_t tiles256 = (size_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (mid_enabled() && N % mid::BNm == 0 && K % mid::BKm == 0 && lda % 8 == 0 && ldw % 8 == 0 &&
      (tiles256 < 128 || (M <= 64 && tiles256 < 512))) {
    static bool attr_mid = false;
    if (!attr_mid) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_mid<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                mid::NSTAGE * mid::STAGE);
      attr_mid = true;
    }
    const int blocks = ((M + mid::BMm - 1) / mid::BMm) * (N / mid::BNm);
    hipLaunchKernelGGL(gemm_nt_mid<EPI>, dim3(blocks), dim3(mid::NTm), mid::NSTAGE * mid::STAGE, s, A, W, C, M, N,
                       K, lda, ldw, ldc, ep);
    FLS_CHECK_LAUNCH();
    return 0;
  }
  int var = variant();
  // the persistent v13 (bit-identical to v10) pays off only where the epilogue is heavy enough to
  // hide the next tile's prologue under it: QKV + RoPE 2.23 -> 2.12 ms on the 70B shape, while the
  // store-only / residual epilogues lose 1-2% to the vmcnt(0) that also waits for the previous
  // tile's store acks (profiles/r1_gemm_persistent)
  if (var == 10 && EPI == FLS_EPI_ROPE && g_rope_persistent) var = 13;
  const bool fast = (N % BN == 0) && (K % BK == 0) && (lda % 8 == 0) && (ldw % 8 == 0) && M > 0;
  // v8/v9 need an even K-tile count (2-tile unrolled body), v9 32-bit X offsets; else v3
  const bool even_k = (K / BK) % 2 == 0;
  if (((var == 9 || var == 10 || var == 11 || var == 12 || var == 13) && !(even_k && (size_t)M * lda * 2 < (1ull << 32))) || (var == 8 && !even_k))
    var = 3;
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  const bool fast4 = fast && (K % (2 * v4::BK4) == 0);
  if (var == 12 && fast) {
    static bool attr12 = false;
    if (!attr12) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_v12<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * v9::BUF);
      attr12 = true;
    }
    hipLaunchKernelGGL(gemm_nt_v12<EPI>, dim3(tiles), dim3(256), 2 * v9::BUF, s, A, W, C, M, N, K, lda, ldw, ldc, ep);
  } else if (var == 11 && fast) {
    static bool attr11 = false;
    if (!attr11) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_v11<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * v9::BUF);
      attr11 = true;
    }
    hipLaunchKernelGGL(gemm_nt_v11<EPI>, dim3(tiles), dim3(256), 2 * v9::BUF, s, A, W, C, M, N, K, lda, ldw, ldc, ep);
  } else if (var == 13 && fast) {
    static bool attr13 = false;
    static int ncu = 256;
    if (!attr13) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_v13<EPI, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * v9::BUF);
      (void)hipFuncSetAttribute((const void*)gemm_nt_v13<EPI, -4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * v9::BUF);
      (void)hipFuncSetAttribute((const void*)gemm_nt_v13<EPI, -8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * v9::BUF);
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) == hipSuccess &&
          hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n >= 8)
        ncu = n & ~7;                            // a multiple of 8: virtual tile ids keep their XCD
      attr13 = true;
    }
    const int grid = tiles < ncu ? tiles : ncu;
    int order = g_v10_order;
    if (order == 0) order = (N / BN <= 64) ? (K >= 16384 ? -4 : -8) : 8;
    if (order == -4)
      hipLaunchKernelGGL((gemm_nt_v13<EPI, -4>), dim3(grid), dim3(256), 2 * v9::BUF, s, A, W, C, M, N, K, lda, ldw,
                         ldc, ep);
    else if (order == -8)
      hipLaunchKernelGGL((gemm_nt_v13<EPI, -8>), dim3(grid), dim3(256), 2 * v9::BUF, s, A, W, C, M, N, K, lda, ldw,
                         ldc, ep);
    else
      hipLaunchKernelGGL((gemm_nt_v13<EPI, 8>), dim3(grid), dim3(256), 2 * v9::BUF, s, A, W, C, M, N, K, lda, ldw,
                         ldc, ep);
  } else if (var == 10 && fast) {
    static bool attr10 = false;
    if (!attr10) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_v10<EPI, 0, 0, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * v9::BUF);
      (void)hipFuncSetAttribute((const void*)gemm_nt_v10<EPI, 0, 0, -4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * v9::BUF);
      (void)hipFuncSetAttribute((const void*)gemm_nt_v10<EPI, 0, 0, -8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * v9::BUF);
      attr10 = true;
    }
    // tile order (scripts/gemm_order.py, profiles/r1_gemm_order): with few N tiles (o / down / qkv
    // projections, N <= 16384) walking M inside groups of N tiles beats the M-grouped order by ~3-4%;
    // the wide gate/up GEMM (N = 57344) keeps 8 M tiles per group
    static const int env_order = [] {
      const char* e = getenv("FLS_GEMM_ORDER");      // A/B of whole runs: 8, -4, -8
      return e ? atoi(e) : 0;
    }();
    int order = g_v10_order ? g_v10_order : env_order;
    if (order == 0) order = (N / BN <= 64) ? (K >= 16384 ? -4 : -8) : 8;
    if (order == -4)
      hipLaunchKernelGGL((gemm_nt_v10<EPI, 0, 0, -4>), dim3(tiles), dim3(256), 2 * v9::BUF, s, A, W, C, M, N, K, lda,
                         ldw, ldc, ep);
    else if (order == -8)
      hipLaunchKernelGGL((gemm_nt_v10<EPI, 0, 0, -8>), dim3(tiles), dim3(256), 2 * v9::BUF, s, A, W, C, M, N, K, lda,
                         ldw, ldc, ep);
    else
      hipLaunchKernelGGL((gemm_nt_v10<EPI, 0, 0, 8>), dim3(tiles), dim3(256), 2 * v9::BUF, s, A, W, C, M, N, K, lda,
                         ldw, ldc, ep);
  } else if (var == 9 && fast) {
    static bool attr9 = false;
    if (!attr9) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_v9<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * v9::BUF);
      attr9 = true;
    }
    hipLaunchKernelGGL(gemm_nt_v9<EPI>, dim3(tiles), dim3(256), 2 * v9::BUF, s, A, W, C, M, N, K, lda, ldw, ldc, ep);
  } else if (var == 8 && fast) {
    static bool attr8 = false;
    if (!attr8) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_v8<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * v7::BUF);
      attr8 = true;
    }
    hipLaunchKernelGGL(gemm_nt_v8<EPI>, dim3(tiles), dim3(512), 2 * v7::BUF, s, A, W, C, M, N, K, lda, ldw, ldc, ep);
  } else if (var == 7 && fast) {
    static bool attr7 = false;
    if (!attr7) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_v7<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * v7::BUF);
      attr7 = true;
    }
    hipLaunchKernelGGL(gemm_nt_v7<EPI>, dim3(tiles), dim3(512), 2 * v7::BUF, s, A, W, C, M, N, K, lda, ldw, ldc, ep);
  } else if (var == 6 && fast) {
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

extern "C" int fls_kernels_version(void) { return 7; }

// v10 tile order: 0 = by shape (default), 8 = M-grouped, -4 / -8 = N-grouped (A/B, tests)
extern "C" int fls_gemm_set_order(int order) {
  if (order != 0 && order != 8 && order != -4 && order != -8) return -1;
  const int old = g_v10_order;
  g_v10_order = order;
  return old;
}

// A/B switch: variant 10's RoPE GEMMs on the persistent v13 kernel (1, default) or on v10 (0)
extern "C" int fls_gemm_set_rope_persistent(int on) {
  const int old = g_rope_persistent;
  g_rope_persistent = on ? 1 : 0;
  return old;
}

// A/B switch for the mid-M kernel (tests / microbenchmarks)
extern "C" int fls_gemm_set_mid(int on) {
  g_mid = on ? 1 : 0;
  return 0;
}

// microbenchmark-only entry: v1 main loop with parts removed (results are garbage)
extern "C" int fls_gemm_ablate(int abl, const void* A, const void* W, void* C, int M, int N, int K,
                               fls_stream_t s) {
  if (N % BN || K % BK) return -2;
  Epi ep{nullptr, 0, nullptr, nullptr, nullptr, 0, 0, nullptr};
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
#define FLS_ABL10_CASE(X)                                                                                    \
  case 40 + X:                                                                                               \
    if ((K / BK) % 2) return -2;                                                                             \
    (void)hipFuncSetAttribute((const void*)gemm_nt_v10<0, X>, hipFuncAttributeMaxDynamicSharedMemorySize,    \
                              2 * v9::BUF);                                                                  \
    hipLaunchKernelGGL((gemm_nt_v10<0, X>), dim3(tiles), dim3(256), 2 * v9::BUF, (hipStream_t)s, a, w, c, M, N, \
                       K, K, K, N, ep);                                                                      \
    break;
    FLS_ABL10_CASE(0) FLS_ABL10_CASE(1) FLS_ABL10_CASE(2) FLS_ABL10_CASE(3) FLS_ABL10_CASE(5) FLS_ABL10_CASE(7)
#undef FLS_ABL10_CASE
#define FLS_SCHED10_CASE(X)                                                                                  \
  case 60 + X:                                                                                               \
    if ((K / BK) % 2) return -2;                                                                             \
    (void)hipFuncSetAttribute((const void*)gemm_nt_v10<0, 0, X>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                              2 * v9::BUF);                                                                  \
    hipLaunchKernelGGL((gemm_nt_v10<0, 0, X>), dim3(tiles), dim3(256), 2 * v9::BUF, (hipStream_t)s, a, w, c, M, N, \
                       K, K, K, N, ep);                                                                      \
    break;
    FLS_SCHED10_CASE(0) FLS_SCHED10_CASE(1) FLS_SCHED10_CASE(2) FLS_SCHED10_CASE(3)
#undef FLS_SCHED10_CASE
    case 70:
    case 71:
      if ((K / BK) % 2) return -2;
      if (abl == 70) {
        (void)hipFuncSetAttribute((const void*)gemm_nt_v12<0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * v9::BUF);
        hipLaunchKernelGGL((gemm_nt_v12<0, 0>), dim3(tiles), dim3(256), 2 * v9::BUF, (hipStream_t)s, a, w, c, M, N, K,
                           K, K, N, ep);
      } else {
        (void)hipFuncSetAttribute((const void*)gemm_nt_v12<0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * v9::BUF);
        hipLaunchKernelGGL((gemm_nt_v12<0, 1>), dim3(tiles), dim3(256), 2 * v9::BUF, (hipStream_t)s, a, w, c, M, N, K,
                           K, K, N, ep);
      }
      break;
#define FLS_ORD10_CASE(X, G)                                                                                 \
  case X:                                                                                                    \
    if ((K / BK) % 2) return -2;                                                                             \
    (void)hipFuncSetAttribute((const void*)gemm_nt_v10<0, 0, 0, G>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                              2 * v9::BUF);                                                                  \
    hipLaunchKernelGGL((gemm_nt_v10<0, 0, 0, G>), dim3(tiles), dim3(256), 2 * v9::BUF, (hipStream_t)s, a, w, c, M, \
                       N, K, K, K, N, ep);                                                                   \
    break;
    FLS_ORD10_CASE(80, 2) FLS_ORD10_CASE(81, 4) FLS_ORD10_CASE(82, 8) FLS_ORD10_CASE(83, 16)
    FLS_ORD10_CASE(84, -4) FLS_ORD10_CASE(85, -8) FLS_ORD10_CASE(86, -16) FLS_ORD10_CASE(87, -2)
    FLS_ORD10_CASE(88, 1) FLS_ORD10_CASE(89, 8)
#undef FLS_ORD10_CASE
    case 50:
      if ((K / BK) % 2) return -2;
      (void)hipFuncSetAttribute((const void*)gemm_nt_v11<0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * v9::BUF);
      hipLaunchKernelGGL((gemm_nt_v11<0, 0>), dim3(tiles), dim3(256), 2 * v9::BUF, (hipStream_t)s, a, w, c, M, N, K,
                         K, K, N, ep);
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
                        int rope_cols, int head_dim, const void* bias, fls_stream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (bias && epi == FLS_EPI_SWIGLU) return -4;
  if ((epi == FLS_EPI_SWIGLU || epi == FLS_EPI_ROPE) && (N % 32)) return -2;
  if (epi == FLS_EPI_ROPE && (head_dim % 32 || rope_cols % 32)) return -3;
  Epi ep{(const half_t*)R, ldr, pos, cos_t, sin_t, rope_cols, head_dim, (const half_t*)bias};
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
