// Skinny-M GEMM (M <= 256: generation steps, small calls) — included by gemm.hip inside its
// anonymous namespace, after splitk_reduce_kernel.
//
// At M = 160 (32 prompts x 5 suffixes, one new row each) a 70B projection is a weight stream: 160
// FLOP per weight byte, 22.9 ms of HBM time per step for 137 GB.  The main / split-K paths pad 160
// rows to 256-row tiles (37.5% of their MFMA and activation-staging work wasted) and ran at
// 3.6-4.5 TB/s (profiles/r3_splitkv).  Here a block is BN = 128 or 256 weight rows (BN / 4 per
// wave: two or four 16-row MFMA subtiles) x ALL of M rounded up to 32 (template RS = 16-row
// subtiles), so every weight byte is read once and no row tile repeats the weight stream:
//   * weights and activations are staged by LDS-DMA (16 B per lane, XOR chunk swizzle on the
//     source address) into a ring of NX stages, DIST = NX - 2 (BN 128) or NX - 1 (BN 256) K-tiles
//     ahead, one counted vmcnt + barrier per K-tile (the mid kernel's scheme; no loop-carried
//     registers but the accumulators);
//   * K is cut into S slices when N / BN blocks leave CUs idle (fp32 partials + the split-K
//     reduce, which applies the epilogue); with S = 1 the NONE / RESID / SWIGLU epilogues run in
//     the kernel (SWIGLU: the first half of each wave's subtiles are gate rows, the second half
//     the matching up rows).
namespace sk {
constexpr int KT = 64;          // K per tile
constexpr int LDS_MAX = 160 * 1024;
// BN = weight rows per block: 128 (two 16-row subtiles per wave) or 256 (four).  At BN = 256 a
// block stages the activations once for twice the weight rows: at M = 160 the activation tile
// (20 KB per K-tile) is larger than a 128-row weight tile (16 KB), and every wave re-reads all of
// it from LDS, so BN = 128 spends more LDS-DMA and LDS-read bytes on the shared activations than
// on the weights it streams.  BN = 256 refills a stage right after the K-tile barrier (LATE: the
// stage freed by that barrier), so NX - 1 K-tiles are in flight from 3 stages of 52 KB.
template <int RS, int BN>
struct Geo {
  static constexpr bool LATE = BN == 256;
  static constexpr int NSUB = BN / 64;                     // 16-row weight subtiles per wave
  static constexpr int XST = RS * 16 * KT * 2;             // activation bytes per stage
  static constexpr int WST = BN * KT * 2;
  static constexpr int STG = XST + WST;
  static constexpr int NX = 4 * STG <= LDS_MAX ? 4 : 3 * STG <= LDS_MAX ? 3 : 2;   // stages
  static constexpr int DIST = LATE ? NX - 1 : NX - 2;      // K-tiles in flight ahead
  static constexpr int QX = RS / 2;                        // 8-row DMA groups per wave: activations
  static constexpr int QW = BN / 32;                       // ... and weights
  static constexpr int LDS = NX * STG;
  static_assert(DIST >= 1, "at least one K-tile in flight");
};
}  // namespace sk

template <int RS, int EPI, int BN>
__global__ __launch_bounds__(256) void gemm_nt_skinny(const half_t* __restrict__ A, const half_t* __restrict__ W,
                                                      half_t* __restrict__ C, int M, int N, int K, int lda, int ldw,
                                                      int ldc, Epi ep) {
  using namespace sk;
  using G = Geo<RS, BN>;
  constexpr int NS = G::NSUB, WR = BN / 4;    // weight subtiles / rows per wave
  static_assert(RS % 2 == 0 && RS >= 2 && RS <= 16, "16-row subtiles: an even count up to 256 rows");
  extern __shared__ __attribute__((aligned(16))) char lds_sk[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, grp = lane >> 4;
  // K slice z of gridDim.y: K-tiles [z * base + min(z, rem), ...), the first rem slices one longer
  // (K = the whole reduction; slices need not divide it)
  const int nkt = K / KT, nsl = (int)gridDim.y, z = (int)blockIdx.y;
  const int nk = nkt / nsl + (z < nkt % nsl ? 1 : 0);                   // K-tiles of this block's slice
  const size_t kofs = (size_t)(z * (nkt / nsl) + min(z, nkt % nsl)) * KT;   // the slice's first K element
  const bool swiglu = EPI == FLS_EPI_SWIGLU;
  // block-local weight row l (wave l / WR, subtile j = (l % WR) / 16) -> physical row; SWIGLU: the
  // first NS / 2 subtiles of a wave are gate rows, the last NS / 2 the matching up rows
  auto phys_row = [&](int l) -> int {
    if (swiglu) {
      const int j = (l % WR) >> 4;
      return (j / (NS / 2)) * ep.gu_rows + (int)blockIdx.x * (BN / 2) + (l / WR) * (WR / 2) + (j % (NS / 2)) * 16 +
             (l & 15);
    }
    return (int)blockIdx.x * BN + l;
  };
  const int cbase = swiglu ? (int)blockIdx.x * (BN / 2) + wave * (WR / 2) : (int)blockIdx.x * BN + wave * WR;

  // LDS-DMA sources: group g = wave + 4 i covers rows 8 g .. 8 g + 7 of its image
  const int sub = lane >> 3;
  const int kc = ((lane & 7) ^ sub) * 8;      // source chunk pre-swizzled (the read XORs it back)
  const half_t* xsrc[G::QX];
  const half_t* wsrc[G::QW];
#pragma unroll
  for (int i = 0; i < G::QX; ++i)
    xsrc[i] = A + kofs + (size_t)min((wave + 4 * i) * 8 + sub, M - 1) * lda + kc;
#pragma unroll
  for (int i = 0; i < G::QW; ++i) wsrc[i] = W + kofs + (size_t)phys_row((wave + 4 * i) * 8 + sub) * ldw + kc;
  auto stage = [&](int t) {
    char* base = lds_sk + (t % G::NX) * G::STG;
#pragma unroll
    for (int i = 0; i < G::QX; ++i) glds16(xsrc[i] + (size_t)t * KT, base + (wave + 4 * i) * 1024);
#pragma unroll
    for (int i = 0; i < G::QW; ++i) glds16(wsrc[i] + (size_t)t * KT, base + G::XST + (wave + 4 * i) * 1024);
  };

  // accumulators pinned in AGPRs and updated in place by asm MFMAs (common.h): compiled MFMAs let
  // the register coalescer rotate the accumulators through copies every K-tile
  floatx4 acc[RS][NS];
#pragma unroll
  for (int i = 0; i < RS; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#define SK_FENCE_ACC()                                                                             \
  _Pragma("unroll") for (int i_ = 0; i_ < RS; ++i_) {                                              \
    _Pragma("unroll") for (int j_ = 0; j_ < NS; ++j_) asm volatile("" : "+a"(acc[i_][j_]));       \
  }
  SK_FENCE_ACC();
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // zero-init VALU writes before the first MFMA

  // DMA is never conditional: past the last tile it re-reads it into a stage nobody reads again,
  // so the vmcnt count is one constant
#pragma unroll
  for (int d = 0; d < G::DIST; ++d) stage(min(d, nk - 1));
  for (int t = 0; t < nk; ++t) {
    if constexpr (!G::LATE) {
      stage(min(t + G::DIST, nk - 1));        // into stage (t + DIST) % NX, last read by tile t - 2
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::DIST * (G::QX + G::QW)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((G::DIST - 1) * (G::QX + G::QW)) : "memory");
    }
    __builtin_amdgcn_s_barrier();             // every wave's part of tile t is in LDS
    // LATE: every wave is past tile t - 1, so its stage ((t + NX - 1) % NX) takes tile t + DIST
    if constexpr (G::LATE) stage(min(t + G::DIST, nk - 1));
    const char* Xs = lds_sk + (t % G::NX) * G::STG;
    const char* Ws = Xs + G::XST;
    // the asm MFMAs are ordered against memory (no read placed after one is hoisted over it), so
    // the schedule is spelled out: K-step 0's fragments, then its MFMAs each followed by one read
    // of K-step 1, whose MFMAs close the tile
    half8 wf[2][NS], xf[2][RS];
    auto rd_w = [&](int s, int j) {
      const int r = wave * WR + j * 16 + fr, c = s * 4 + grp;
      wf[s][j] = *(const half8*)(Ws + r * 128 + ((c ^ (r & 7)) << 4));
    };
    auto rd_x = [&](int s, int i) {
      const int r = i * 16 + fr, c = s * 4 + grp;
      xf[s][i] = *(const half8*)(Xs + r * 128 + ((c ^ (r & 7)) << 4));
    };
#pragma unroll
    for (int j = 0; j < NS; ++j) rd_w(0, j);
#pragma unroll
    for (int i = 0; i < RS; ++i) rd_x(0, i);
#pragma unroll
    for (int j = 0; j < NS; ++j) rd_w(1, j);
#pragma unroll
    for (int i = 0; i < RS; ++i) {
#pragma unroll
      for (int j = 0; j < NS; ++j) mfma_acc_inplace_ordered(acc[i][j], wf[0][j], xf[0][i]);
      rd_x(1, i);
    }
#pragma unroll
    for (int i = 0; i < RS; ++i)
#pragma unroll
      for (int j = 0; j < NS; ++j) mfma_acc_inplace_ordered(acc[i][j], wf[1][j], xf[1][i]);
  }
  // the tail's redundant DMA must land before this block's LDS can be handed to another block;
  // the accumulators were written by MFMAs the hazard recognizer cannot see
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  SK_FENCE_ACC();
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#undef SK_FENCE_ACC

  // epilogue: lane holds columns cbase + 16 j + 4 grp + r of row 16 i + fr
#pragma unroll
  for (int i = 0; i < RS; ++i) {
    const int m = i * 16 + fr;
    if (m >= M) continue;
    const float rsc = row_scale(ep, m);
    if constexpr (EPI == EPI_F32) {           // split-K partial slab of this slice (ldc = N floats)
      float* Cf = (float*)C + (size_t)blockIdx.y * ep.part_stride + (size_t)m * ldc;
#pragma unroll
      for (int j = 0; j < NS; ++j) *(floatx4*)(Cf + cbase + 16 * j + 4 * grp) = acc[i][j];
    } else if constexpr (EPI == FLS_EPI_SWIGLU) {
#pragma unroll
      for (int j = 0; j < NS / 2; ++j) {
        half4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (half_t)(silu(acc[i][j][r] * rsc) * (acc[i][j + NS / 2][r] * rsc));
        *(half4*)(C + (size_t)m * ldc + cbase + 16 * j + 4 * grp) = o;
      }
    } else {
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        const int n = cbase + 16 * j + 4 * grp;
        floatx4 a = acc[i][j] * rsc;
        if (ep.bias) {
          const half4 b = *(const half4*)(ep.bias + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) a[r] += (float)b[r];
        }
        if constexpr (EPI == FLS_EPI_RESID) {
          const half4 rr = *(const half4*)(ep.R + (size_t)m * ep.ldr + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) a[r] = a[r] * ep.alpha + (float)rr[r];
        }
        half4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (half_t)a[r];
        *(half4*)(C + (size_t)m * ldc + n) = o;
      }
    }
  }
}

int g_skinny = 1;            // skinny-M path: 0 off, 1 auto, 2 any M <= 256 it supports (tests / A-B)
int g_skinny_blocks = 0;     // K split: 0 = the BN's rule (try_skinny), n = until N / BN x S >= n (A/B)
int g_skinny_bn = 0;         // weight rows per block: 0 auto, 128 / 256 forced where supported (A/B)

template <int EPI, int RS, int BN>
int launch_skinny_rs(const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda, int ldw, int ldc,
                     const Epi& ep, hipStream_t s, int S) {
  static bool attr = false;
  constexpr int lds = sk::Geo<RS, BN>::LDS;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_nt_skinny<RS, EPI, BN>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              lds);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_nt_skinny<RS, EPI, BN>), dim3(N / BN, S), dim3(256), lds, s, A, W, C, M, N, K, lda, ldw,
                     ldc, ep);
  FLS_CHECK_LAUNCH();
  return 0;
}

// BN = 256 is instantiated for RS <= 10 (M <= 160): from RS = 12 on only two 56+ KB stages fit
constexpr int SK_BN256_MAX_RS = 10;

template <int EPI>
int launch_skinny_epi(int rs, int bn, const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda,
                      int ldw, int ldc, const Epi& ep, hipStream_t s, int S) {
  if (bn == 256) {
    switch (rs) {
      case 2: return launch_skinny_rs<EPI, 2, 256>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
      case 4: return launch_skinny_rs<EPI, 4, 256>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
      case 6: return launch_skinny_rs<EPI, 6, 256>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
      case 8: return launch_skinny_rs<EPI, 8, 256>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
      default: return launch_skinny_rs<EPI, 10, 256>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    }
  }
  switch (rs) {
    case 2: return launch_skinny_rs<EPI, 2, 128>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    case 4: return launch_skinny_rs<EPI, 4, 128>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    case 6: return launch_skinny_rs<EPI, 6, 128>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    case 8: return launch_skinny_rs<EPI, 8, 128>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    case 10: return launch_skinny_rs<EPI, 10, 128>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    case 12: return launch_skinny_rs<EPI, 12, 128>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    case 14: return launch_skinny_rs<EPI, 14, 128>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    default: return launch_skinny_rs<EPI, 16, 128>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
  }
}

// -> 1 when the skinny path took the GEMM, 0 when it does not apply, < 0 on a launch error
template <int EPI>
int try_skinny(const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda, int ldw, int ldc,
               const Epi& ep, hipStream_t s, void* ws, size_t ws_bytes) {
  if (!g_skinny || M > 256 || N % 128 || K % sk::KT || lda % 8 || ldw % 8 || ((uintptr_t)A & 15) ||
      ((uintptr_t)W & 15))
    return 0;
  const int rs = ((M + 31) / 32) * 2;
  const int nkt = K / sk::KT;
  // auto: the measured range (profiles/r4_gen, 70B shapes): M 17..192 on the narrow projections;
  // the wide gate/up GEMM (N / 128 >= 256 blocks, 224 main-path tiles) runs faster on the main
  // path at M = 64 / 160 / 256 (175 / 209 / 221 us vs 195 / 246 / 332 with 128-row blocks), but at
  // 65..144 rows the 256-row block without a K split beats it (same box, M = 96 / 112 / 128 / 144:
  // 180 / 182 / 184 / 199 us vs 216 / 205 / 199 / 206; profiles/r4_gen/gateup_mid_m)
  const bool wide = N / 128 >= 256;
  const bool wide_bn256 = wide && M > 64 && M <= 144 && N % 256 == 0;
  if (g_skinny == 1 && (M < 17 || M > 192 || (wide && !wide_bn256))) return 0;
  // K slices.  BN = 128: else the fewest powers of two that give whole 256-CU rounds or at least
  // two rounds (one block per CU: a fractional single round leaves a tail of full-K blocks).  BN = 256: the fewest that give 192 blocks (3/4 of
  // the CUs; its deeper DMA queue keeps HBM busy from fewer CUs).  g_skinny_blocks > 0 (A/B) sets
  // a block target instead.
  // BN = 128 first tries one round of 7/8 to all of the CUs with uneven slices (70B QKV at M = 160:
  // 80 blocks x 3 = 240 instead of 80 x 8 = 640, 2.5 rounds, and 8 slabs of fp32 partials).
  auto slices = [&](int bn) {
    const long nblk = N / bn;
    if (bn == 128 && g_skinny_blocks == 0) {
      for (int s = 2; s <= 16 && nblk * s <= 256; ++s)
        if (nblk * s >= 224 && nkt / s >= 8) return s;
    }
    auto good = [&](int s) {
      const long b = nblk * s;
      if (g_skinny_blocks > 0) return b >= g_skinny_blocks;
      return bn == 256 ? b >= 192 : (b % 256 == 0 || b >= 512);
    };
    int s = 1;
    while (!good(s) && s < 16 && nkt % (2 * s) == 0 && nkt / (2 * s) >= 8) s *= 2;
    return s;
  };
  // BN = 256 (auto) where its split gives whole 256-CU rounds: the 70B O and down projections
  // (32 x 8 blocks), 4% faster on down at M = 160 and equal on O; QKV (40 x 8) and gate/up (224 x 1)
  // run slower with it (profiles/r4_gen/bn256/skinny_ab.log)
  const bool bn256_ok = N % 256 == 0 && rs <= SK_BN256_MAX_RS;
  int bn = 128;
  if (bn256_ok && (g_skinny_bn == 256 ||
                   (g_skinny_bn == 0 && (wide_bn256 || (long)(N / 256) * slices(256) % 256 == 0))))
    bn = 256;
  const int S = slices(bn);
  const bool direct_epi = EPI == FLS_EPI_NONE || EPI == FLS_EPI_RESID || EPI == FLS_EPI_SWIGLU;
  const bool direct = S == 1 && direct_epi;
  if (direct) {
    if (ldc % 4 || ((uintptr_t)C & 7)) return 0;
    if (EPI == FLS_EPI_RESID && (ep.ldr % 4 || ((uintptr_t)ep.R & 7))) return 0;
    const int rc =
        launch_skinny_epi<direct_epi ? EPI : FLS_EPI_NONE>(rs, bn, A, W, C, M, N, K, lda, ldw, ldc, ep, s, 1);
    return rc ? rc : 1;
  }
  // fp32 partial slabs + the split-K reduce (applies the epilogue)
  if (!ws || ((uintptr_t)ws & 15) || (size_t)S * M * N * 4 > ws_bytes || ldc % 4 || ((uintptr_t)C & 7) ||
      (EPI == FLS_EPI_RESID && (ep.ldr % 4 || ((uintptr_t)ep.R & 7))))
    return 0;
  Epi e = ep;
  e.part_stride = (long long)M * N;
  float* part = (float*)ws;
  int rc = launch_skinny_epi<EPI_F32>(rs, bn, A, W, (half_t*)part, M, N, K, lda, ldw, N, e, s, S);
  if (rc) return rc;
  const long long threads = (long long)M * (N / 4);
  hipLaunchKernelGGL(splitk_reduce_kernel<EPI>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, part, S,
                     e.part_stride, M, N, C, ldc, e);
  FLS_CHECK_LAUNCH();
  return 1;
}
