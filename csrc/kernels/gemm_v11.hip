// gemm_nt_v11: the 70B projection GEMM on a 384 x 256 x 64 tile (gfx950 / MI355X).
//
//   C[M, N'] = epilogue( A[M, K] . W[N, K]^T )      fp16 in, fp32 accumulate  (same contract as gemm.hip)
//
// Why a bigger tile.  v10 (256 x 256 x 64, gemm_v10.h) moves 64 KiB through LDS-DMA per 8.4 MFLOP
// K-tile: at the full MFMA rate that is 32 B/clk/CU of L2 -> LDS traffic, the per-CU LDS-DMA ceiling
// (profiles/r2_gemm: the same loop with the DMA bytes dropped runs +47-54%).  The tile is capped by
// the accumulators: 4 waves x 128 x 128 fp32 = all 256 AGPRs of every wave.  v11 keeps 4 waves (one per
// SIMD, 512 registers each) and gives each wave 192 x 128 outputs: 256 accumulators in AGPRs (row
// groups 0..7) + 128 in arch VGPRs (row groups 8..11).  Per K-tile: 80 KiB for 12.6 MFLOP = 26.7 B/clk
// at the full MFMA rate (-17% bytes per FLOP), and the two 80 KiB stages fill the CU's 160 KiB LDS.
//
// Register budget (arch VGPRs): 128 accumulators + ONE k-step of operand fragments (12 x 8 = 20
// half8 = 80 VGPRs; v10 holds two k-steps) + addresses.  The fragments are refilled in place right
// after their last MFMA of the k-step, so the read-ahead distance is one k-step (96 MFMAs) for x rows
// 0..7 and w, and half a k-step for x rows 8..11.
//
// Schedule.  One K-tile = two k-steps (s0, s1) x three phases of 32 MFMAs:
//   A: x rows 0..3 x w 0..7 (row-major)  -- refills x[0..3] for the next k-step, reads x[8..9] of this one
//   B: x rows 4..7 x w 0..7 (row-major)  -- refills x[4..7], reads x[10..11]
//   C: x rows 8..11 x w 0..7 (column-major) -- refills w[0..7]
// LDS regions per stage: X0 / X1 / X2 = stage rows {0..63, 192..255} / {64..127, 256..319} /
// {128..191, 320..383} (16 KiB each; the two wave rows of a region), W (32 KiB).  Phases pair into
// super-phases SP0 = (A s0, B s0), SP1 = (C s0, A s1), SP2 = (B s1, C s1), each ending in a relaxed
// lgkmcnt (LDS reads retire in order) + counted vmcnt + raw s_barrier.  Region r of a stage is refilled (tile t -> t+2) in an SP after
// the barrier that follows its last read.  LDS-DMA plan per wave:
//   SP0 of tile t: X2(t+1), W half 2 (t+1)          (4 + 4 pieces)   end: lgkmcnt(6) vmcnt(16)
//   SP1 of tile t: X0(t+2)                          (4 pieces)       end: lgkmcnt(6) vmcnt(4)
//   SP2 of tile t: X1(t+2), W half 1 (t+2)          (4 + 4 pieces)   end: lgkmcnt(8) vmcnt(12)
// (W half h = each wave's DMA groups 4h-4 .. 4h-1 of its 8.)
// (+0-1.5% over 4 / 4 / 12 pieces with all of W(t+2) in SP2 on the four 70B shapes,
// profiles/r4_gemm/variant_ab_s2_a1.log.)  Requires an even number of K-tiles (the loop body is unrolled over both stages) and M >= 384: the last M tile is shifted
// back to end at row M and stores only the rows its neighbour does not (epilogue_quadrant's LO), so
// every LDS-DMA source row is in bounds and the per-piece row offsets live in the scalar soffset.
#include "gemm_v10.h"


namespace {
namespace v11 {
constexpr int TM = 384, TN = 256, TK = 64;
// LDS (160 KiB, the whole CU): per stage b an X01 image (x row groups 0..7 of both wave rows,
// 256 rows x 128 B), an X2 image (row groups 8..11, 128 rows) and a W image (256 rows), laid out
// [X01 0][X01 1][X2 0][X2 1][W 0][W 1] so that every fragment read is one of 6 per-lane base
// registers (image x k-step) + an immediate offset < 64 KiB (stage, row group).  Rows are 128 B
// with the XOR chunk swizzle (chunk c of row r in slot c ^ (r & 7)).
constexpr int X01_0 = 0, X01_STG = 32768;
constexpr int X2_0 = 65536, X2_STG = 16384;
constexpr int W_0 = 98304, W_STG = 32768;
constexpr int LDS_BYTES = 163840;
}  // namespace v11

// accumulate into an arch-VGPR accumulator (row groups 8..11); same ordering contract as
// mfma_acc_inplace_ordered (common.h)
__device__ __forceinline__ void mfma_acc_v_ordered(floatx4& c, const half8& a, const half8& b) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b) : "memory");
}

template <int EPI>
__global__ __launch_bounds__(256, 1) void gemm_nt_v11(const half_t* __restrict__ A, const half_t* __restrict__ W,
                                                    half_t* __restrict__ C, int M, int N, int K, int lda, int ldw,
                                                    int ldc, Epi ep) {
  using namespace v11;
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
  const int tiles_m = (M + TM - 1) / TM;
  const int tiles_n = N / TN;
  const int2 tmn = tile_of(bid, tiles_m, tiles_n, ep.order);
  const int mlo = tmn.x * TM;                 // first row this block stores
  const int m0 = min(mlo, M - TM);            // rows computed: [m0, m0 + TM)
  const int n0 = tmn.y * TN;

  // LDS-DMA: a piece = 8 rows x 128 B; lane l moves row l>>3, global chunk (l&7)^(l>>3) into slot l&7
  const int lr = lane >> 3;
  const int lc = (lane & 7) ^ lr;
  const unsigned xl = (unsigned)(lr * lda + lc * 8) * 2u;
  const unsigned wl = (unsigned)(lr * ldw + lc * 8) * 2u;
  const char* Ab = (const char*)(A + (size_t)m0 * lda);
  const char* Wb = (const char*)(W + (size_t)(EPI == FLS_EPI_SWIGLU ? n0 / 2 : n0) * ldw);
  // descriptors over A / W; past the last K-tile a DMA goes through the same base with 0 records
  // (issued and counted by vmcnt, moves no bytes): only the num_records word is selected per tile
  auto rsrc = [](const char* base, bool live) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, live ? -1 : 0, 0x00020000);
  };
  // wave-uniform pieces: X region j (0..2), piece i (0..3): LDS byte offset and source row
  // (regions 0 / 1 = x row groups 0..3 / 4..7 of the X01 image, 2 = the X2 image); W piece i (0..7)
  int xlds_p[3][4];
  unsigned xso[3][4];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = 4 * wave + i;
      const int src_row = (p >> 3) * 192 + j * 64 + (p & 7) * 8;
      xlds_p[j][i] = j < 2 ? X01_0 + ((p >> 3) * 128 + j * 64 + (p & 7) * 8) * 128
                           : X2_0 + ((p >> 3) * 64 + (p & 7) * 8) * 128;
      xso[j][i] = (unsigned)(src_row * lda) * 2u;
    }
  unsigned wso[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int l = (8 * wave + i) * 8;
    const int pr = EPI == FLS_EPI_SWIGLU ? ((l >> 4) & 1) * ep.gu_rows + (l >> 5) * 16 + (l & 15) : l;
    wso[i] = (unsigned)(pr * ldw) * 2u;
  }
#define V11_DMA_X(rs, buf, j, i, k0)                                                               \
  __builtin_amdgcn_raw_ptr_buffer_load_lds(                                                        \
      rs, (LDS_AS void*)(smem + xlds_p[j][i] + (buf) * ((j) < 2 ? X01_STG : X2_STG)), 16, xl,      \
      xso[j][i] + (unsigned)(k0) * 2u, 0, 0)
#define V11_DMA_W(rs, buf, i, k0)                                                                  \
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)(smem + W_0 + (buf) * W_STG + (8 * wave + (i)) * 1024), \
                                           16, wl, wso[i] + (unsigned)(k0) * 2u, 0, 0)

  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, grp = lane >> 4;
  const int sw = fr & 7;
  const int cs0 = ((0 + grp) ^ sw) << 4;
  const int cs1 = ((4 + grp) ^ sw) << 4;
  const int xrow = X01_0 + (wm * 128 + fr) * 128;
  const int x2row = X2_0 + (wm * 64 + fr) * 128;
  const int wrow = W_0 + (wn * 128 + fr) * 128;

  // row groups 0..7: AGPR accumulators; 8..11: arch-VGPR accumulators
  floatx4 acc[8][8], accv[4][8];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int t = 0; t < 8; ++t) accv[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  half8 xf[12], wf[8];
#define V11_FENCE_ACC()                                                                            \
  _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_)                                                \
  _Pragma("unroll") for (int t_ = 0; t_ < 8; ++t_) asm volatile("" : "+a"(acc[u_][t_]));          \
  _Pragma("unroll") for (int u_ = 0; u_ < 4; ++u_)                                                \
  _Pragma("unroll") for (int t_ = 0; t_ < 8; ++t_) asm volatile("" : "+v"(accv[u_][t_]));
  V11_FENCE_ACC();
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");

  // the 6 per-lane fragment base addresses (image x k-step); everything else is an immediate
  const char* const bx01_0 = smem + xrow + cs0;
  const char* const bx01_1 = smem + xrow + cs1;
  const char* const bx2_0 = smem + x2row + cs0;
  const char* const bx2_1 = smem + x2row + cs1;
  const char* const bw_0 = smem + wrow + cs0;
  const char* const bw_1 = smem + wrow + cs1;
#define V11_RX(f, buf, s)                                                                          \
  xf[f] = (f) < 8 ? *(const half8*)(((s) ? bx01_1 : bx01_0) + (buf) * X01_STG + (f) * 2048)        \
                  : *(const half8*)(((s) ? bx2_1 : bx2_0) + (buf) * X2_STG + ((f) - 8) * 2048)
#define V11_RW(t, buf, s) wf[t] = *(const half8*)(((s) ? bw_1 : bw_0) + (buf) * W_STG + (t) * 2048)
#define V11_MFMA(u, t)                                                                             \
  do {                                                                                            \
    if ((u) < 8) mfma_acc_inplace_ordered(acc[(u) & 7][t], wf[t], xf[u]);                         \
    else mfma_acc_v_ordered(accv[(u) & 3][t], wf[t], xf[u]);                                      \
  } while (0)
// DMA slots of a phase with ND (2, 4 or 6) DMAs: after these MFMAs
#define V11_DMA_AT(i_, ND)                                                                         \
  ((ND) == 2 ? ((i_) == 9 ? 0 : (i_) == 21 ? 1 : -1)                                              \
   : (ND) == 4 ? ((i_) == 7 ? 0 : (i_) == 13 ? 1 : (i_) == 19 ? 2 : (i_) == 25 ? 3 : -1)          \
   : ((i_) == 5 ? 0 : (i_) == 9 ? 1 : (i_) == 13 ? 2 : (i_) == 17 ? 3 : (i_) == 21 ? 4 : (i_) == 25 ? 5 : -1))
#define V11_DMAS(i_, DMA_STMT, ND)                                                                 \
  {                                                                                               \
    const int d_ = V11_DMA_AT(i_, ND);                                                            \
    if (d_ >= 0) { DMA_STMT(d_); }                                                                \
  }
// End of a super-phase: retire this wave's LDS reads except the LGK youngest (all of them read
// regions that the next SP does not refill; LDS reads complete in order), this wave's DMAs except
// the VMC youngest, then the barrier.
#define V11_SYNC(LGK, VMC)                                                                         \
  {                                                                                               \
    __builtin_amdgcn_s_waitcnt(0xC07F | ((LGK) << 8));                                            \
    asm volatile("s_waitcnt vmcnt(" #VMC ")" ::: "memory");                                       \
    __builtin_amdgcn_s_barrier();                                                                 \
  }

// Phase A: x rows 0..3 x w 0..7, column-major (w column t first used at MFMA 4t, so the w
// refills of the preceding C phase have ~29 MFMAs to land).  After MFMA 1 / 3 read x rows 8 / 9
// of the current k-step (cbuf, cs); after the last use of x row u (MFMA 28 + u) refill it with
// the next k-step (nbuf, ns).
#define V11_PHASE_A(cbuf, cs, nbuf, ns, DMA_STMT, ND)                                             \
  _Pragma("unroll") for (int i_ = 0; i_ < 32; ++i_) {                                             \
    const int t_ = i_ >> 2, u_ = i_ & 3;                                                          \
    V11_MFMA(u_, t_);                                                                             \
    if (i_ == 1) V11_RX(8, cbuf, cs);                                                             \
    if (i_ == 3) V11_RX(9, cbuf, cs);                                                             \
    if (i_ >= 28) V11_RX(u_, nbuf, ns);                                                           \
    V11_DMAS(i_, DMA_STMT, ND);                                                                   \
  }
// Phase B: x rows 4..7 x w 0..7, row-major; reads x rows 10 / 11 of the current k-step after
// MFMAs 1 / 3 and refills x row u after its last MFMA (8u' + 7).
#define V11_PHASE_B(cbuf, cs, nbuf, ns, DMA_STMT, ND)                                             \
  _Pragma("unroll") for (int i_ = 0; i_ < 32; ++i_) {                                             \
    const int u_ = 4 + (i_ >> 3), t_ = i_ & 7;                                                    \
    V11_MFMA(u_, t_);                                                                             \
    if (i_ == 1) V11_RX(10, cbuf, cs);                                                            \
    if (i_ == 3) V11_RX(11, cbuf, cs);                                                            \
    if ((i_ & 7) == 7) V11_RX(u_, nbuf, ns);                                                      \
    V11_DMAS(i_, DMA_STMT, ND);                                                                   \
  }
// Phase C: x rows 8..11 x w 0..7, column-major; refills w column t after its last MFMA (4t + 3).
#define V11_PHASE_C(nbuf, ns, DMA_STMT, ND)                                                       \
  _Pragma("unroll") for (int i_ = 0; i_ < 32; ++i_) {                                             \
    const int t_ = i_ >> 2, u_ = 8 + (i_ & 3);                                                    \
    V11_MFMA(u_, t_);                                                                             \
    if ((i_ & 3) == 3) V11_RW(t_, nbuf, ns);                                                      \
    V11_DMAS(i_, DMA_STMT, ND);                                                                   \
  }

  const int nk = K / TK;                       // even (host-checked)
  // prologue: tile 0 (X0 X1 W X2) and tile 1 (X0 X1 W), then retire tile 0 and read the k-step
  // (0, s0) fragments of x rows 0..7 and w.  In steady state, at the end of SP2 of tile t-1 the
  // DMAs in flight are X0(t+1) (SP1) and X1 W(t+1) (SP2): 16 per wave.
  const __amdgpu_buffer_rsrc_t rA = rsrc(Ab, true), rW = rsrc(Wb, true);
  const __amdgpu_buffer_rsrc_t rZA = rsrc(Ab, false), rZW = rsrc(Wb, false);
  {
    const int k1 = min(1, nk - 1) * TK;
#pragma unroll
    for (int i = 0; i < 4; ++i) V11_DMA_X(rA, 0, 0, i, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) V11_DMA_X(rA, 0, 1, i, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) V11_DMA_W(rW, 0, i, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) V11_DMA_X(rA, 0, 2, i, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) V11_DMA_X(rA, 1, 0, i, k1);
#pragma unroll
    for (int i = 0; i < 4; ++i) V11_DMA_X(rA, 1, 1, i, k1);
#pragma unroll
    for (int i = 0; i < 4; ++i) V11_DMA_W(rW, 1, i, k1);     // W-lo(1); W-hi(1) in SP0 of tile 0
  }
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int u = 0; u < 8; ++u) V11_RX(u, 0, 0);
#pragma unroll
  for (int t = 0; t < 8; ++t) V11_RW(t, 0, 0);

  for (int kt = 0; kt < nk; kt += 2) {
    const int k1 = min(kt + 1, nk - 1) * TK, k2 = min(kt + 2, nk - 1) * TK, k3 = min(kt + 3, nk - 1) * TK;
    const __amdgpu_buffer_rsrc_t rX1 = kt + 1 < nk ? rA : rZA;
    const __amdgpu_buffer_rsrc_t rX2 = kt + 2 < nk ? rA : rZA, rW2 = kt + 2 < nk ? rW : rZW;
    const __amdgpu_buffer_rsrc_t rX3 = kt + 3 < nk ? rA : rZA, rW3 = kt + 3 < nk ? rW : rZW;
    // DMA plan of tile t (stage b = t & 1), 8 / 4 / 8 DMAs per super-phase (W split: W-lo(t+2) in
    // SP2 of tile t, W-hi(t+2) in SP0 of tile t+1, waited at the end of SP1 of tile t+1 with
    // everything older):
    //   SP0: X2(t+1) + W-hi(t+1) -> b^1   lgkmcnt(6) vmcnt(16)
    //   SP1: X0(t+2) -> b                 lgkmcnt(6) vmcnt(4)
    //   SP2: X1(t+2) + W-lo(t+2) -> b     lgkmcnt(8) vmcnt(12)
    const __amdgpu_buffer_rsrc_t rW1 = kt + 1 < nk ? rW : rZW;
#define V11_TILE(B, rXn, rWn, kn, rXf, rWf, kf)                                                    \
  {                                                                                               \
    auto dX2 = [&](int d) { V11_DMA_X(rXn, (B) ^ 1, 2, d, kn); };                                 \
    auto dWhi = [&](int d) { V11_DMA_W(rWn, (B) ^ 1, d + 4, kn); };                               \
    auto dX0a = [&](int d) { V11_DMA_X(rXf, B, 0, d, kf); };                                      \
    auto dX0b = [&](int d) { V11_DMA_X(rXf, B, 0, d + 2, kf); };                                  \
    auto dX1 = [&](int d) { V11_DMA_X(rXf, B, 1, d, kf); };                                       \
    auto dWlo = [&](int d) { V11_DMA_W(rWf, B, d, kf); };                                         \
    V11_PHASE_A(B, 0, B, 1, dX2, 4);                     /* A s0 */                              \
    V11_PHASE_B(B, 0, B, 1, dWhi, 4);                    /* B s0 */                              \
    V11_SYNC(6, 16);                                     /* SP0 */                               \
    V11_PHASE_C(B, 1, dX0a, 2);                          /* C s0 */                              \
    V11_PHASE_A(B, 1, (B) ^ 1, 0, dX0b, 2);              /* A s1 */                              \
    V11_SYNC(6, 4);                                      /* SP1 */                               \
    V11_PHASE_B(B, 1, (B) ^ 1, 0, dX1, 4);               /* B s1 */                              \
    V11_PHASE_C((B) ^ 1, 0, dWlo, 4);                    /* C s1 */                              \
    V11_SYNC(8, 12);                                     /* SP2 */                               \
  }
    V11_TILE(0, rX1, rW1, k1, rX2, rW2, k2);   // tile kt,   stage 0
    V11_TILE(1, rX2, rW2, k2, rX3, rW3, k3);   // tile kt+1, stage 1
#undef V11_TILE
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  V11_FENCE_ACC();
#undef V11_FENCE_ACC
#undef V11_RX
#undef V11_RW
#undef V11_MFMA
#undef V11_DMA_AT
#undef V11_DMAS
#undef V11_SYNC
#undef V11_PHASE_A
#undef V11_PHASE_B
#undef V11_PHASE_C
#undef V11_DMA_X
#undef V11_DMA_W

  const int mrow = m0 + wm * 192 + fr, ncol = n0 + wn * 128;
  // VGPR row groups first (frees their 128 registers before the AGPR ones are read out)
  epilogue_quadrant<EPI, 4, true>(C, ldc, M, mrow + 128, ncol, grp, accv, ep, mlo);
  epilogue_quadrant<EPI, 8, true>(C, ldc, M, mrow, ncol, grp, acc, ep, mlo);
}

int g_v11 = 1;               // 0 off, 1 auto (v11_pays), 2 any valid shape (tests)
// time of one 384 x 256 v11 tile in 256 x 256 v10 tiles, x 100 (v11_pays)
int g_v11_cost = 145;

// Whole 256-CU tile rounds of each kernel at this shape, a v11 tile priced at g_v11_cost / 100
// v10 tiles: a launch whose tile count is not a multiple of 256 pays its last round in full.
// (Replaces the rule "no more padded rows than v10", which sent 14,784-row micro-batches to v10's
// 8 rounds instead of v11's 5 and 16,128 rows to v11's 6 instead of v10's 8:
// profiles/r5_resident/gemm_m.log.)  v10
// runs rows past its ROW_CHUNK (gemm.hip; default 16384) as evenly sized launches, each with its
// own tail.
bool v11_pays(int M, int N) {
  using namespace v11;
  const long t11 = (long)((M + TM - 1) / TM) * (N / TN);
  const long r11 = (t11 + 255) / 256;
  const int n_chunks = M > 16384 ? (M + 16383) / 16384 : 1;
  const int step = ((M + n_chunks - 1) / n_chunks + 255) / 256 * 256;
  long r10 = 0;
  for (int r0 = 0; r0 < M; r0 += step) {
    const long t10 = (long)((min(step, M - r0) + 255) / 256) * (N / 256);
    r10 += (t10 + 255) / 256;
  }
  return r11 * g_v11_cost <= r10 * 100;
}

template <int EPI>
int launch_v11(const half_t* A, const half_t* W, half_t* C, int M, int N, int K, int lda, int ldw, int ldc, Epi ep,
               hipStream_t s) {
  using namespace v11;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_nt_v11<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    attr = true;
  }
  const int tiles_m = (M + TM - 1) / TM, tiles_n = N / TN;
  ep.order = auto_order(tiles_m, tiles_n);
  hipLaunchKernelGGL((gemm_nt_v11<EPI>), dim3(tiles_m * tiles_n), dim3(256), LDS_BYTES, s, A, W, C, M, N, K, lda, ldw,
                     ldc, ep);
  FLS_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// 0 = v10 everywhere, 1 = v11 where it takes no more whole tile rounds (default), 2 = v11 on every
// shape it supports (tests: small and ragged shapes); returns the previous mode
extern "C" int fls_gemm_set_v11(int mode) {
  const int old = g_v11;
  g_v11 = mode < 0 ? 0 : mode > 2 ? 2 : mode;
  return old;
}

// 1 when the auto mode prices v11 at or below v10 for an M x N launch (host-side rule, tests)
extern "C" int fls_gemm_v11_pays(int M, int N) { return v11_pays(M, N) ? 1 : 0; }

// the auto mode's price of a v11 tile in v10 tiles x 100 (<= 0: keep); returns the previous price
extern "C" int fls_gemm_set_v11_cost(int cost) {
  const int old = g_v11_cost;
  if (cost > 0) g_v11_cost = cost;
  return old;
}

// Applicability of v11 for a launch; the shape rules of gemm.hip's v10 main path plus M >= 384.
// Called from fls_gemm (gemm.hip) before its own dispatch.  Returns 1 and launches when v11 takes
// the GEMM, 0 when it does not apply, < 0 on a launch error.
extern "C" int fls_gemm_v11_try(const void* A, const void* W, void* C, const void* R, int M, int N, int K, int lda,
                                int ldw, int ldc, int ldr, int epi, const int* pos, const float* cos_t,
                                const float* sin_t, int rope_cols, int head_dim, const void* bias,
                                const float* rscale, float alpha, float* ss, int ss_ld, fls_stream_t s) {
  using namespace v11;
  if (!g_v11 || M < TM || N % TN || K % TK || (K / TK) % 2 || lda % 8 || ldw % 8) return 0;
  if (g_v11 == 1) {
    // fills the chip (at least one tile per CU per launch) and takes no longer in whole tile rounds
    if ((size_t)((M + TM - 1) / TM) * (N / TN) < 256 || !v11_pays(M, N)) return 0;
  }
  // 32-bit DMA offsets: every row of A (piece rows + lane rows + K) and of the (stacked) weight
  if ((size_t)M * lda * 2 >= (1ull << 32)) return 0;
  if (epi == FLS_EPI_SWIGLU && (size_t)(N / 2 + TN) * ldw * 2 >= (1ull << 32)) return 0;
  if ((size_t)N * ldw * 2 >= (1ull << 32)) return 0;
  // 16-byte epilogue stores / residual loads
  if (ldc % 8 || ((uintptr_t)C & 15)) return 0;
  if (epi == FLS_EPI_RESID && (ldr % 8 || ((uintptr_t)R & 15))) return 0;
  Epi ep{(const half_t*)R, ldr, pos, cos_t, sin_t, rope_cols, head_dim, (const half_t*)bias, N / 2, 0,
         nullptr, nullptr, nullptr, 0, 0};
  ep.rs = rscale;
  ep.alpha = alpha;
  ep.ss = ss;
  ep.ss_ld = ss_ld;
  auto a = (const half_t*)A;
  auto w = (const half_t*)W;
  auto c = (half_t*)C;
  auto st = (hipStream_t)s;
  int rc;
  switch (epi) {
    case FLS_EPI_NONE: rc = launch_v11<FLS_EPI_NONE>(a, w, c, M, N, K, lda, ldw, ldc, ep, st); break;
    case FLS_EPI_RESID: rc = launch_v11<FLS_EPI_RESID>(a, w, c, M, N, K, lda, ldw, ldc, ep, st); break;
    case FLS_EPI_SWIGLU: rc = launch_v11<FLS_EPI_SWIGLU>(a, w, c, M, N, K, lda, ldw, ldc, ep, st); break;
    case FLS_EPI_ROPE:
      rc = head_dim == 128 ? launch_v11<FLS_EPI_ROPE>(a, w, c, M, N, K, lda, ldw, ldc, ep, st)
                           : launch_v11<EPI_ROPE64>(a, w, c, M, N, K, lda, ldw, ldc, ep, st);
      break;
    default: return 0;
  }
  return rc ? rc : 1;
}
