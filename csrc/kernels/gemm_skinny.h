// Skinny-M GEMM (M <= 256: generation steps, small calls) — included by gemm.hip inside its
// anonymous namespace, after splitk_reduce_kernel.
//
// At M = 160 (32 prompts x 5 suffixes, one new row each) a 70B projection is a weight stream: 160
// FLOP per weight byte, 22.9 ms of HBM time per step for 137 GB.  The main / split-K paths pad 160
// rows to 256-row tiles (37.5% of their MFMA and activation-staging work wasted) and ran at
// 3.6-4.5 TB/s (profiles/r3_splitkv).  Here a block is 128 weight rows (32 per wave: two 16-row
// MFMA subtiles) x ALL of M rounded up to 32 (template RS = 16-row subtiles), so every weight byte
// is read once and no row tile repeats the weight stream:
//   * weights and activations are staged by LDS-DMA (16 B per lane, XOR chunk swizzle on the
//     source address) into a ring of NX stages, DIST = NX - 2 K-tiles ahead, one counted vmcnt +
//     barrier per K-tile (the mid kernel's scheme; no loop-carried registers but the accumulators);
//   * K is cut into S slices when N / 128 blocks leave CUs idle (fp32 partials + the split-K
//     reduce, which applies the epilogue); with S = 1 the NONE / RESID / SWIGLU epilogues run in
//     the kernel (SWIGLU: each wave's two subtiles are matching gate and up rows).
namespace sk {
constexpr int BNW = 128;        // weight rows per block
constexpr int KT = 64;          // K per tile
constexpr int WST = BNW * KT * 2;
constexpr int LDS_MAX = 160 * 1024;
template <int RS>
struct Geo {
  static constexpr int XST = RS * 16 * KT * 2;             // activation bytes per stage
  static constexpr int STG = XST + WST;
  static constexpr int NX = 4 * STG <= LDS_MAX ? 4 : 3;    // stages
  static constexpr int DIST = NX - 2;                      // K-tiles in flight ahead
  static constexpr int QX = RS / 2;                        // 8-row DMA groups per wave: activations
  static constexpr int QW = BNW / 32;                      // ... and weights
  static constexpr int LDS = NX * STG;
};
}  // namespace sk

template <int RS, int EPI>
__global__ __launch_bounds__(256) void gemm_nt_skinny(const half_t* __restrict__ A, const half_t* __restrict__ W,
                                                      half_t* __restrict__ C, int M, int N, int K, int lda, int ldw,
                                                      int ldc, Epi ep) {
  using namespace sk;
  using G = Geo<RS>;
  static_assert(RS % 2 == 0 && RS >= 2 && RS <= 16, "16-row subtiles: an even count up to 256 rows");
  extern __shared__ __attribute__((aligned(16))) char lds_sk[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, grp = lane >> 4;
  const int nk = K / KT;                      // K-tiles of this block's slice
  const size_t kofs = (size_t)blockIdx.y * K; // the slice's first K element
  const bool swiglu = EPI == FLS_EPI_SWIGLU;
  // block-local weight row l (wave l / 32, subtile (l / 16) & 1) -> physical row; SWIGLU: subtile 0
  // = gate rows, subtile 1 = the matching up rows
  auto phys_row = [&](int l) -> int {
    if (swiglu) return ((l >> 4) & 1) * ep.gu_rows + (int)blockIdx.x * (BNW / 2) + (l >> 5) * 16 + (l & 15);
    return (int)blockIdx.x * BNW + l;
  };
  const int cbase = swiglu ? (int)blockIdx.x * (BNW / 2) + wave * 16 : (int)blockIdx.x * BNW + wave * 32;

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
  floatx4 acc[RS][2];
#pragma unroll
  for (int i = 0; i < RS; ++i) acc[i][0] = acc[i][1] = floatx4{0.f, 0.f, 0.f, 0.f};
#define SK_FENCE_ACC()                                                                             \
  _Pragma("unroll") for (int i_ = 0; i_ < RS; ++i_) {                                              \
    asm volatile("" : "+a"(acc[i_][0]));                                                           \
    asm volatile("" : "+a"(acc[i_][1]));                                                           \
  }
  SK_FENCE_ACC();
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // zero-init VALU writes before the first MFMA

  // DMA is never conditional: past the last tile it re-reads it into a stage nobody reads again,
  // so the vmcnt count is one constant
#pragma unroll
  for (int d = 0; d < G::DIST; ++d) stage(min(d, nk - 1));
  for (int t = 0; t < nk; ++t) {
    stage(min(t + G::DIST, nk - 1));          // into stage (t + DIST) % NX, last read by tile t - 2
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::DIST * (G::QX + G::QW)) : "memory");
    __builtin_amdgcn_s_barrier();             // every wave's part of tile t is in LDS
    const char* Xs = lds_sk + (t % G::NX) * G::STG;
    const char* Ws = Xs + G::XST;
    // the asm MFMAs are ordered against memory (no read placed after one is hoisted over it), so
    // the schedule is spelled out: K-step 0's fragments, then its MFMAs each followed by one read
    // of K-step 1, whose MFMAs close the tile
    half8 wf[2][2], xf[2][RS];
    auto rd_w = [&](int s, int j) {
      const int r = wave * 32 + j * 16 + fr, c = s * 4 + grp;
      wf[s][j] = *(const half8*)(Ws + r * 128 + ((c ^ (r & 7)) << 4));
    };
    auto rd_x = [&](int s, int i) {
      const int r = i * 16 + fr, c = s * 4 + grp;
      xf[s][i] = *(const half8*)(Xs + r * 128 + ((c ^ (r & 7)) << 4));
    };
    rd_w(0, 0);
    rd_w(0, 1);
#pragma unroll
    for (int i = 0; i < RS; ++i) rd_x(0, i);
    rd_w(1, 0);
    rd_w(1, 1);
#pragma unroll
    for (int i = 0; i < RS; ++i) {
      mfma_acc_inplace_ordered(acc[i][0], wf[0][0], xf[0][i]);
      mfma_acc_inplace_ordered(acc[i][1], wf[0][1], xf[0][i]);
      rd_x(1, i);
    }
#pragma unroll
    for (int i = 0; i < RS; ++i) {
      mfma_acc_inplace_ordered(acc[i][0], wf[1][0], xf[1][i]);
      mfma_acc_inplace_ordered(acc[i][1], wf[1][1], xf[1][i]);
    }
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
    if constexpr (EPI == EPI_F32) {           // split-K partial slab of this slice (ldc = N floats)
      float* Cf = (float*)C + (size_t)blockIdx.y * ep.part_stride + (size_t)m * ldc;
#pragma unroll
      for (int j = 0; j < 2; ++j) *(floatx4*)(Cf + cbase + 16 * j + 4 * grp) = acc[i][j];
    } else if constexpr (EPI == FLS_EPI_SWIGLU) {
      half4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (half_t)(silu(acc[i][0][r]) * acc[i][1][r]);
      *(half4*)(C + (size_t)m * ldc + cbase + 4 * grp) = o;
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = cbase + 16 * j + 4 * grp;
        floatx4 a = acc[i][j];
        if (ep.bias) {
          const half4 b = *(const half4*)(ep.bias + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) a[r] += (float)b[r];
        }
        if constexpr (EPI == FLS_EPI_RESID) {
          const half4 rr = *(const half4*)(ep.R + (size_t)m * ep.ldr + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) a[r] += (float)rr[r];
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
int g_skinny_blocks = 0;     // K split: 0 = whole-round rule (try_skinny), n = until N / 128 x S >= n (A/B)

template <int EPI, int RS>
int launch_skinny_rs(const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda, int ldw, int ldc,
                     const Epi& ep, hipStream_t s, int S) {
  static bool attr = false;
  constexpr int lds = sk::Geo<RS>::LDS;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_nt_skinny<RS, EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_nt_skinny<RS, EPI>), dim3(N / sk::BNW, S), dim3(256), lds, s, A, W, C, M, N, K / S, lda,
                     ldw, ldc, ep);
  FLS_CHECK_LAUNCH();
  return 0;
}

template <int EPI>
int launch_skinny_epi(int rs, const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda, int ldw,
                      int ldc, const Epi& ep, hipStream_t s, int S) {
  switch (rs) {
    case 2: return launch_skinny_rs<EPI, 2>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    case 4: return launch_skinny_rs<EPI, 4>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    case 6: return launch_skinny_rs<EPI, 6>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    case 8: return launch_skinny_rs<EPI, 8>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    case 10: return launch_skinny_rs<EPI, 10>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    case 12: return launch_skinny_rs<EPI, 12>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    case 14: return launch_skinny_rs<EPI, 14>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
    default: return launch_skinny_rs<EPI, 16>(A, W, C, M, N, K, lda, ldw, ldc, ep, s, S);
  }
}

// -> 1 when the skinny path took the GEMM, 0 when it does not apply, < 0 on a launch error
template <int EPI>
int try_skinny(const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda, int ldw, int ldc,
               const Epi& ep, hipStream_t s, void* ws, size_t ws_bytes) {
  if (!g_skinny || M > 256 || N % sk::BNW || K % sk::KT || lda % 8 || ldw % 8 || ((uintptr_t)A & 15) ||
      ((uintptr_t)W & 15))
    return 0;
  const int nblk = N / sk::BNW, nkt = K / sk::KT;
  // auto: the measured range (profiles/r4_gen, 70B shapes): M 17..192 on the narrow projections;
  // the wide gate/up GEMM (N / 128 >= 256 blocks, 224 main-path tiles) runs faster on the main
  // path at every M measured (64 / 160 / 256 rows: 175 / 209 / 221 us vs 195 / 246 / 332)
  if (g_skinny == 1 && (M < 17 || M > 192 || nblk >= 256)) return 0;
  // K slices: the fewest that give whole 256-CU rounds or at least two rounds (one block per CU:
  // a fractional single round leaves a tail of full-K blocks; 70B at M = 160: O / down S = 4,
  // QKV S = 8 measured fastest); g_skinny_blocks > 0 (A/B) sets a block target instead
  int S = 1;
  auto good = [&](int s) {
    const long b = (long)nblk * s;
    return g_skinny_blocks > 0 ? b >= g_skinny_blocks : (b % 256 == 0 || b >= 512);
  };
  while (!good(S) && S < 16 && nkt % (2 * S) == 0 && nkt / (2 * S) >= 8) S *= 2;
  const bool direct_epi = EPI == FLS_EPI_NONE || EPI == FLS_EPI_RESID || EPI == FLS_EPI_SWIGLU;
  const bool direct = S == 1 && direct_epi;
  const int rs = ((M + 31) / 32) * 2;
  if (direct) {
    if (ldc % 4 || ((uintptr_t)C & 7)) return 0;
    if (EPI == FLS_EPI_RESID && (ep.ldr % 4 || ((uintptr_t)ep.R & 7))) return 0;
    const int rc = launch_skinny_epi<direct_epi ? EPI : FLS_EPI_NONE>(rs, A, W, C, M, N, K, lda, ldw, ldc, ep, s, 1);
    return rc ? rc : 1;
  }
  // fp32 partial slabs + the split-K reduce (applies the epilogue)
  if (!ws || ((uintptr_t)ws & 15) || (size_t)S * M * N * 4 > ws_bytes || ldc % 4 || ((uintptr_t)C & 7) ||
      (EPI == FLS_EPI_RESID && (ep.ldr % 4 || ((uintptr_t)ep.R & 7))))
    return 0;
  Epi e = ep;
  e.part_stride = (long long)M * N;
  float* part = (float*)ws;
  int rc = launch_skinny_epi<EPI_F32>(rs, A, W, (half_t*)part, M, N, K, lda, ldw, N, e, s, S);
  if (rc) return rc;
  const long long threads = (long long)M * (N / 4);
  hipLaunchKernelGGL(splitk_reduce_kernel<EPI>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, part, S,
                     e.part_stride, M, N, C, ldc, e);
  FLS_CHECK_LAUNCH();
  return 1;
}
