// Panel GEMM (row-exact small M: generation steps) — included by gemm.hip inside its anonymous
// namespace, after gemm_nt_mid.
//
// A reused generation step runs row-exact (every output row gets the arithmetic the full pass
// gave it), which rules out K splits: each output element is ONE accumulator chain over K in
// ascending 64-wide tiles, the v10 / v11 / mid order.  At small M the mid kernel's 64 x 128
// tiles leave the narrow projections with few blocks (70B O / down at M <= 64: 64).  Here a block
// is ALL of M (up to 64 RT rows) x 32 output columns:
//   * the N / 32 blocks each stream their 32 weight rows once (70B O / down: 256 blocks, QKV 320,
//     gate/up 1792) while the activations (M x K, shared by every block) come from L2;
//   * 4 waves split the rows (16-row tiles u = wave + 4 i), each against both 16-column subtiles,
//     so a wave's fragments are the mid kernel's: the same MFMA (16x16x32 f16), the same K chunk
//     per lane group, the same ascending K order -> bitwise the mid / v10 / v11 result per row;
//   * operands by LDS-DMA (16 B per lane, XOR chunk swizzle on the source) into a 3-deep ring,
//     one counted vmcnt + barrier per K-tile (the mid kernel's scheme);
//   * the epilogues are the mid kernel's helpers (store_pair_off / store_rope_pair), so they round
//     the same way; RoPE blocks take a head's columns j*16.. and their partners j*16 + hd/2.
namespace pn {
constexpr int KT = 64, PBN = 32, NST = 3;
template <int RT>
struct Geo {
  static constexpr int MP = 64 * RT;                 // rows staged (M rounded up to 64 RT)
  static constexpr int XST = MP * KT * 2;            // activation bytes per stage
  static constexpr int STG = XST + PBN * KT * 2;
  static constexpr int QX = RT * 2;                  // 8-row DMA groups per wave (activations)
  static constexpr int Q = QX + 1;                   // ... + one weight group per wave
  static constexpr int LDS = NST * STG;
  static_assert(LDS <= 160 * 1024, "LDS");
};
constexpr int MAX_RT = 5;                            // M <= 320
}  // namespace pn

template <int RT, int EPI>
__global__ __launch_bounds__(256) void gemm_nt_panel(const half_t* __restrict__ A, const half_t* __restrict__ W,
                                                     half_t* __restrict__ C, int M, int N, int K, int lda, int ldw,
                                                     int ldc, Epi ep) {
  using namespace pn;
  using G = Geo<RT>;
  extern __shared__ __attribute__((aligned(16))) char lds_pn[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, grp = lane >> 4;
  const int b = blockIdx.x, nk = K / KT;
  // first output column of this block's two 16-column subtiles (RoPE: a pair of partner columns)
  int c0 = b * PBN, c1 = b * PBN + 16;
  if constexpr (is_rope(EPI)) {
    const int half = ep.head_dim >> 1, per = half >> 4;
    c0 = (b / per) * ep.head_dim + (b % per) * 16;
    c1 = c0 + half;
  }
  // LDS-DMA sources.  Activation group g = wave + 4 i: rows 8 g .. 8 g + 7 (clamped to M - 1);
  // weight group `wave`: rows 8 (wave & 1) .. + 7 of subtile wave >> 1
  const int sub = lane >> 3;
  const int kc = ((lane & 7) ^ sub) * 8;             // source chunk pre-swizzled (the read XORs it back)
  const half_t* xsrc[G::QX];
#pragma unroll
  for (int i = 0; i < G::QX; ++i) xsrc[i] = A + (size_t)min((wave + 4 * i) * 8 + sub, M - 1) * lda + kc;
  const int wl = (wave & 1) * 8 + sub;
  int wrow = ((wave >> 1) ? c1 : c0) + wl;
  if constexpr (EPI == FLS_EPI_SWIGLU) wrow = gu_phys_row(b * PBN + (wave >> 1) * 16 + wl, ep.gu_rows);
  const half_t* wsrc = W + (size_t)wrow * ldw + kc;
  auto stage = [&](int kt) {
    char* base = lds_pn + (kt % NST) * G::STG;
#pragma unroll
    for (int i = 0; i < G::QX; ++i) glds16(xsrc[i] + (size_t)kt * KT, base + (wave + 4 * i) * 1024);
    glds16(wsrc + (size_t)kt * KT, base + G::XST + wave * 1024);
  };

  floatx4 acc[RT][2];
#pragma unroll
  for (int i = 0; i < RT; ++i) acc[i][0] = acc[i][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  bool live[RT];                                     // this wave's 16-row tiles holding rows < M
#pragma unroll
  for (int i = 0; i < RT; ++i) live[i] = (wave + 4 * i) * 16 < M;

  stage(0);
  if (nk > 1) stage(1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 2 < nk) {
      stage(kt + 2);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G::Q) : "memory");   // tiles kt+1, kt+2 in flight
    } else if (kt + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::Q) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();                    // every wave's part of tile kt landed
    const char* Xs = lds_pn + (kt % NST) * G::STG;
    const char* Ws = Xs + G::XST;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + grp;                    // logical 16-byte chunk of this lane
      half8 wf[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int r = t * 16 + fr;
        wf[t] = *(const half8*)(Ws + r * 128 + ((c ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < RT; ++i) {
        if (!live[i]) continue;                      // wave-uniform
        const int r = (wave + 4 * i) * 16 + fr;
        const half8 xf = *(const half8*)(Xs + r * 128 + ((c ^ (r & 7)) << 4));
        acc[i][0] = mfma16x16x32(wf[0], xf, acc[i][0]);
        acc[i][1] = mfma16x16x32(wf[1], xf, acc[i][1]);
      }
    }
    // WAR: stage(kt + 3) (next iteration) overwrites this buffer; all reads are done
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
#pragma unroll
  for (int i = 0; i < RT; ++i) {
    const int m = (wave + 4 * i) * 16 + fr;
    if (m >= M) continue;
    if constexpr (is_rope(EPI)) {
      store_rope_pair(C, ldc, m, c0 + 4 * grp, acc[i][0], acc[i][1], ep);
    } else {
      store_pair_off<EPI>(C, ldc, m, b * PBN, 4 * grp, acc[i][0], acc[i][1], ep);
    }
  }
}

int g_panel = 1;             // panel path: 0 off, 1 row-exact calls where it wins, 2 every M <= 320 it takes (A/B)

template <int EPI, int RT>
void launch_panel_rt(const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda, int ldw, int ldc,
                     const Epi& ep, hipStream_t s) {
  static bool attr = false;
  constexpr int lds = pn::Geo<RT>::LDS;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_nt_panel<RT, EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_nt_panel<RT, EPI>), dim3(N / pn::PBN), dim3(256), lds, s, A, W, C, M, N, K, lda, ldw, ldc,
                     ep);
}

// -> 1 when the panel path took the GEMM, 0 when it does not apply
template <int EPI>
int try_panel(const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda, int ldw, int ldc,
              const Epi& ep, hipStream_t s) {
  if (!g_panel || (g_panel == 1 && !ep.row_exact)) return 0;
  // auto (1): where it measured faster than the mid kernel, row-exact 70B shapes (profiles/r6_decode,
  // scripts/decode_gemm_bench.py): M = 64 QKV 52.6 vs 61.1 us, O 51.1 vs 60.0, down 170 vs 231; not the wide
  // gate/up (234 vs 171) nor any shape at M = 160 / 320 (2.5x slower: every block stages ALL the
  // activation rows, so the L2 -> LDS activation traffic is N / 32 times M x K and bounds it)
  if (g_panel == 1 && (M > 64 || N > 16384)) return 0;
  if (M < 1 || M > 64 * pn::MAX_RT || N % pn::PBN || K % pn::KT || lda % 8 || ldw % 8 || ((uintptr_t)A & 15) ||
      ((uintptr_t)W & 15) || ldc % 4 || ((uintptr_t)C & 7))
    return 0;
  if (EPI == FLS_EPI_RESID && (ep.ldr % 4 || ((uintptr_t)ep.R & 7))) return 0;
  if (is_rope(EPI) && (ep.head_dim % 32 || N % ep.head_dim)) return 0;
  if (EPI == FLS_EPI_SWIGLU && ep.gu_rows * 2 != N) return 0;
  switch ((M + 63) / 64) {
    case 1: launch_panel_rt<EPI, 1>(A, W, C, M, N, K, lda, ldw, ldc, ep, s); break;
    case 2: launch_panel_rt<EPI, 2>(A, W, C, M, N, K, lda, ldw, ldc, ep, s); break;
    case 3: launch_panel_rt<EPI, 3>(A, W, C, M, N, K, lda, ldw, ldc, ep, s); break;
    case 4: launch_panel_rt<EPI, 4>(A, W, C, M, N, K, lda, ldw, ldc, ep, s); break;
    default: launch_panel_rt<EPI, 5>(A, W, C, M, N, K, lda, ldw, ldc, ep, s); break;
  }
  return 1;
}
