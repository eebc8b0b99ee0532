// Sparse mixture-of-experts FFN on gfx950 (Mixtral, Qwen3-MoE).
//
// Per MLP chunk of T tokens (h = post-attention RMSNorm output, x = residual stream):
//   1. router logits   [T, E]  = h . Wr^T                     (fls_gemm, fp16 out like HF's Linear)
//   2. fls_moe_route   one wave per token: fp32 softmax over E, top-k (ties -> lower expert id),
//                      optional renormalisation, -> ids [T*k], weights [T*k] (fp32; Qwen3-MoE rounds
//                      them to fp16 like HF)
//   3. fls_moe_plan    one workgroup: stable counting sort of the T*k (token, slot) entries by expert
//                      -> offs [E+1] (rows of each expert in the permuted order), tiles [E+1] (their
//                      256-row GEMM tiles, prefix), rows [T*k] (permuted row -> token), dest [T*k]
//                      (entry -> permuted row).  Deterministic: entries keep token order inside an
//                      expert, so a run is bitwise reproducible.
//   4. fls_moe_gemm    the v10 MFMA GEMM in grouped form (gemm_v10.h): every expert's rows in ONE
//                      launch, no host round trip for the counts.  gate/up + SwiGLU gathers its A rows
//                      straight from h through `rows` (the LDS-DMA source offsets are per row, fixed
//                      for the whole K loop, so the gather costs one index load per staged row); down
//                      reads the permuted SwiGLU output contiguously.
//   5. fls_moe_combine x[t] += sum_j w[t,j] * y[dest[t,j]] in the rounding of HF's expert loop: each
//                      contribution rounded to fp16, accumulated in fp16 in ascending expert order,
//                      then added to the residual (transformers MixtralExperts / Qwen3MoeExperts).
// Reference: the reference runs any AutoModelForCausalLM with the model.layers.N layout
// (/root/reference/utils.py:101-115); these kernels give the MoE families a native path.
#include "gemm_v10.h"

namespace {

constexpr int ROUTE_WAVES = 4;
constexpr int PLAN_THREADS = 1024;
constexpr int PLAN_WAVES = PLAN_THREADS / WAVE;
constexpr int MAX_E = 256;
constexpr int MAX_K = 8;

__device__ __forceinline__ void wave_argmax(float& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(i, o, 64);
    if (ov > v || (ov == v && oi < i)) {
      v = ov;
      i = oi;
    }
  }
}

// one wave per token; lane j holds experts j, j+64, j+128, j+192
__global__ __launch_bounds__(ROUTE_WAVES * 64) void moe_route_kernel(const half_t* __restrict__ logits, int ldl,
                                                                     int T, int E, int k, int norm, int round16,
                                                                     int* __restrict__ ids, float* __restrict__ w) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * ROUTE_WAVES + (threadIdx.x >> 6);
  if (t >= T) return;
  float l[4];
  float mx = -INFINITY;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = lane + 64 * q;
    l[q] = e < E ? (float)logits[(size_t)t * ldl + e] : -INFINITY;
    mx = fmaxf(mx, l[q]);
  }
  mx = warp_max(mx);
  float p[4], s = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    p[q] = lane + 64 * q < E ? __expf(l[q] - mx) : 0.f;
    s += p[q];
  }
  s = warp_sum(s);
  const float inv = 1.f / s;
  // top-k by k rounds of a wave argmax (constant-indexed arrays: registers, not scratch)
  float sel_p[MAX_K];
  int sel_i[MAX_K];
  float tot = 0.f;
#pragma unroll
  for (int j = 0; j < MAX_K; ++j) {
    if (j >= k) break;
    float v = -1.f;
    int vi = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = lane + 64 * q;
      if (e < E && p[q] >= 0.f && (p[q] > v || (p[q] == v && e < vi))) {
        v = p[q];
        vi = e;
      }
    }
    wave_argmax(v, vi);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (lane + 64 * q == vi) p[q] = -1.f;               // taken
    sel_p[j] = v * inv;
    sel_i[j] = vi;
    tot += sel_p[j];
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < MAX_K; ++j) {
      if (j >= k) break;
      float wj = norm ? sel_p[j] / tot : sel_p[j];
      if (round16) wj = (float)(half_t)wj;
      ids[(size_t)t * k + j] = sel_i[j];
      w[(size_t)t * k + j] = wj;
    }
  }
}

// single workgroup: stable counting sort of n entries by expert id
__global__ __launch_bounds__(PLAN_THREADS) void moe_plan_kernel(const int* __restrict__ ids, int n, int k, int E,
                                                                int* __restrict__ offs, int* __restrict__ tiles,
                                                                int* __restrict__ rows, int* __restrict__ dest) {
  __shared__ int hist[PLAN_WAVES][MAX_E];
  __shared__ int off[MAX_E + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < PLAN_WAVES * MAX_E; i += PLAN_THREADS) (&hist[0][0])[i] = 0;
  __syncthreads();
  const int chunk = (n + PLAN_WAVES - 1) / PLAN_WAVES;
  const int lo = min(n, wave * chunk), hi = min(n, lo + chunk);
  for (int i = lo + lane; i < hi; i += 64) atomicAdd(&hist[wave][ids[i]], 1);
  __syncthreads();
  if (tid < E) {                      // per expert: exclusive prefix over the waves' chunks
    int run = 0;
    for (int v = 0; v < PLAN_WAVES; ++v) {
      const int c = hist[v][tid];
      hist[v][tid] = run;
      run += c;
    }
    off[tid + 1] = run;               // count, scanned below
  }
  __syncthreads();
  if (tid == 0) {
    off[0] = 0;
    int t = 0;
    offs[0] = 0;
    tiles[0] = 0;
    for (int e = 0; e < E; ++e) {
      const int c = off[e + 1];
      off[e + 1] = off[e] + c;
      t += (c + BM - 1) / BM;
      offs[e + 1] = off[e + 1];
      tiles[e + 1] = t;
    }
  }
  __syncthreads();
  // each wave walks its chunk in order, 64 entries at a time: rank among the group's earlier
  // lanes with the same expert, then the last lane of each expert advances that expert's base
  for (int g0 = lo; g0 < hi; g0 += 64) {
    const int i = g0 + lane;
    const int id = i < hi ? ids[i] : -1;
    int before = 0, after = 0;
    for (int j = 0; j < 64; ++j) {
      const int o = __shfl(id, j, 64);
      before += (j < lane && o == id) ? 1 : 0;
      after += (j > lane && o == id) ? 1 : 0;
    }
    if (id >= 0) {
      const int pos = off[id] + hist[wave][id] + before;
      dest[i] = pos;
      rows[pos] = i / k;
    }
    __builtin_amdgcn_wave_barrier();
    if (id >= 0 && after == 0) hist[wave][id] += before + 1;
    __builtin_amdgcn_wave_barrier();
  }
}

// x[t] = fp16(x[t] + acc), acc = fp16 sum over the token's slots in ascending expert order of
// fp16(y[dest] * w); one block per token row, 8 columns (16 B) per thread and step
__global__ __launch_bounds__(256) void moe_combine_kernel(const half_t* __restrict__ y, int ldy,
                                                          const int* __restrict__ ids, const int* __restrict__ dest,
                                                          const float* __restrict__ w, half_t* __restrict__ x, int ldx,
                                                          int k, int H) {
  const int t = blockIdx.x;
  // the token's k experts are distinct: slot j goes in place rank_j of the ascending-id order
  int id[MAX_K], order[MAX_K];
#pragma unroll
  for (int j = 0; j < MAX_K; ++j) id[j] = j < k ? ids[(size_t)t * k + j] : 0x7fffffff;
#pragma unroll
  for (int r = 0; r < MAX_K; ++r) {
    int sel = 0;
#pragma unroll
    for (int j = 0; j < MAX_K; ++j) {
      int rank = 0;
#pragma unroll
      for (int i = 0; i < MAX_K; ++i) rank += (id[i] < id[j] || (id[i] == id[j] && i < j)) ? 1 : 0;
      sel = rank == r ? j : sel;
    }
    order[r] = sel;
  }
  for (int c = threadIdx.x * 8; c < H; c += blockDim.x * 8) {
    half8 acc = {};
#pragma unroll
    for (int r = 0; r < MAX_K; ++r) {
      if (r >= k) break;
      const int e = t * k + order[r];
      const float wj = w[e];
      const half8 v = *(const half8*)(y + (size_t)dest[e] * ldy + c);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = (half_t)((float)acc[q] + (float)(half_t)((float)v[q] * wj));
    }
    half8 xv = *(const half8*)(x + (size_t)t * ldx + c);
#pragma unroll
    for (int q = 0; q < 8; ++q) xv[q] = (half_t)((float)xv[q] + (float)acc[q]);
    *(half8*)(x + (size_t)t * ldx + c) = xv;
  }
}

template <int EPI>
int launch_grouped(const half_t* A, const half_t* W, half_t* C, int M_bound, int N, int K, int lda, int ldw,
                   int ldc, const int* tiles, const int* offs, const int* rows, int n_groups, long long wstride,
                   hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_nt_v10<EPI, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * BUF);
    attr = true;
  }
  const int tiles_m = (M_bound + BM - 1) / BM, tiles_n = N / BN;
  Epi ep{nullptr, 0, nullptr, nullptr, nullptr, 0, 0, nullptr, N / 2, auto_order(tiles_m, tiles_n),
         tiles, offs, rows, wstride, n_groups};
  hipLaunchKernelGGL((gemm_nt_v10<EPI, true>), dim3(tiles_m * tiles_n), dim3(256), 2 * BUF, s, A, W, C, M_bound, N,
                     K, lda, ldw, ldc, ep);
  FLS_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int fls_moe_route(const void* logits, int ldl, int T, int E, int k, int norm, int round16, int* ids,
                             float* w, fls_stream_t s) {
  if (T <= 0) return 0;
  if (E < 1 || E > MAX_E || k < 1 || k > MAX_K || k > E) return -2;
  hipLaunchKernelGGL(moe_route_kernel, dim3((T + ROUTE_WAVES - 1) / ROUTE_WAVES), dim3(ROUTE_WAVES * 64), 0,
                     (hipStream_t)s, (const half_t*)logits, ldl, T, E, k, norm, round16, ids, w);
  FLS_CHECK_LAUNCH();
  return 0;
}

extern "C" int fls_moe_plan(const int* ids, int n, int k, int E, int* offs, int* tiles, int* rows, int* dest,
                            fls_stream_t s) {
  if (E < 1 || E > MAX_E || k < 1 || n < 0) return -2;
  hipLaunchKernelGGL(moe_plan_kernel, dim3(1), dim3(PLAN_THREADS), 0, (hipStream_t)s, ids, n, k, E, offs, tiles,
                     rows, dest);
  FLS_CHECK_LAUNCH();
  return 0;
}

extern "C" int fls_moe_combine(const void* y, int ldy, const int* ids, const int* dest, const float* w, void* x,
                               int ldx, int T, int k, int H, fls_stream_t s) {
  if (T <= 0) return 0;
  if (k < 1 || k > MAX_K || H % 8 || ldx % 8 || ldy % 8) return -2;
  hipLaunchKernelGGL(moe_combine_kernel, dim3(T), dim3(256), 0, (hipStream_t)s, (const half_t*)y, ldy, ids, dest, w,
                     (half_t*)x, ldx, k, H);
  FLS_CHECK_LAUNCH();
  return 0;
}

// Grouped expert GEMM (v10 grouped form).  epi: FLS_EPI_SWIGLU (W per group = [gate; up], C has N/2
// columns) or FLS_EPI_NONE.  rows: optional gather (A row of each permuted row), else A is permuted.
// M_bound >= sum over groups of their rows rounded up to 256 (T*k + 255*G suffices).  Returns -5 when
// the shape is outside the kernel's contract (caller falls back to per-group fls_gemm).
extern "C" int fls_moe_gemm(const void* A, const void* W, void* C, int M_bound, int N, int K, int lda, int ldw,
                            int ldc, int epi, const int* tiles, const int* offs, const int* rows, int n_groups,
                            long long wstride, int a_rows, fls_stream_t s) {
  if (M_bound <= 0) return 0;
  const bool ok = N % BN == 0 && K % BK == 0 && (K / BK) % 2 == 0 && lda % 8 == 0 && ldw % 8 == 0 && ldc % 8 == 0 &&
                  ((uintptr_t)C & 15) == 0 && n_groups >= 1 && n_groups <= MAX_E &&
                  (size_t)a_rows * lda * 2 < (1ull << 32) &&
                  (size_t)(epi == FLS_EPI_SWIGLU ? N / 2 + BN : N) * ldw * 2 < (1ull << 32) &&
                  (epi == FLS_EPI_SWIGLU || epi == FLS_EPI_NONE);
  if (!ok) return -5;
  auto a = (const half_t*)A;
  auto w = (const half_t*)W;
  auto c = (half_t*)C;
  auto st = (hipStream_t)s;
  if (epi == FLS_EPI_SWIGLU)
    return launch_grouped<FLS_EPI_SWIGLU>(a, w, c, M_bound, N, K, lda, ldw, ldc, tiles, offs, rows, n_groups, wstride,
                                          st);
  return launch_grouped<FLS_EPI_NONE>(a, w, c, M_bound, N, K, lda, ldw, ldc, tiles, offs, rows, n_groups, wstride, st);
}
