// Sparse mixture-of-experts FFN on gfx950 (Mixtral, Qwen3-MoE, Qwen2-MoE).
//
// Per MLP chunk of T tokens (h = post-attention RMSNorm output, x = residual stream):
//   1. router logits   [T, E]  = h . Wr^T                     (fls_gemm, fp16 out like HF's Linear)
//   2. fls_moe_route   one wave per token: fp32 softmax over E, top-k (ties -> lower expert id),
//                      optional renormalisation, -> ids [T*k], weights [T*k] (fp32; Qwen3-MoE rounds
//                      them to fp16 like HF)
//   3. fls_moe_plan    stable counting sort of the T*k (token, slot) entries by expert (3 launches)
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

// softmax over the token's E logits (lane j holds experts j, j+64, j+128, j+192 in l[]), top-k by k
// rounds of a wave argmax (ties -> lower id), optional renormalisation / fp16 rounding; lane 0 writes
__device__ __forceinline__ void route_token(const float (&l)[4], int lane, int E, int k, int norm, int round16,
                                            size_t t, int* __restrict__ ids, float* __restrict__ w) {
  float mx = -INFINITY;
#pragma unroll
  for (int q = 0; q < 4; ++q) mx = fmaxf(mx, l[q]);
  mx = warp_max(mx);
  float p[4], s = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    p[q] = lane + 64 * q < E ? __expf(l[q] - mx) : 0.f;
    s += p[q];
  }
  s = warp_sum(s);
  const float inv = 1.f / s;
  // constant-indexed arrays: registers, not scratch
  float sel_p[MAX_K];
  int sel_i[MAX_K];
  float tot = 0.f;
#pragma unroll
  for (int j = 0; j < MAX_K; ++j) {
    if (j >= k) continue;
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
      if (j >= k) continue;
      float wj = norm ? sel_p[j] / tot : sel_p[j];
      if (round16) wj = (float)(half_t)wj;
      ids[t * k + j] = sel_i[j];
      w[t * k + j] = wj;
    }
  }
}

// routing from fp16 logits [T, E] (E > 64: the logits come from the mid-M GEMM); one wave per token
__global__ __launch_bounds__(ROUTE_WAVES * 64) void moe_route_kernel(const half_t* __restrict__ logits, int ldl,
                                                                     int T, int E, int k, int norm, int round16,
                                                                     int* __restrict__ ids, float* __restrict__ w) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * ROUTE_WAVES + (threadIdx.x >> 6);
  if (t >= T) return;
  float l[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = lane + 64 * q;
    l[q] = e < E ? (float)logits[(size_t)t * ldl + e] : -INFINITY;
  }
  route_token(l, lane, E, k, norm, round16, t, ids, w);
}

// router logits + routing for E <= EMAX (<= 64): TPW tokens per wave, each lane owning 16-byte column
// chunks lane*8 + 512 i of the hidden dimension; every router-row chunk loaded once per wave feeds
// the TPW tokens.  The logits are summed over the wave, rounded to fp16 (HF's router Linear runs in
// the activation dtype) and handed to route_token.  Replaces an N = E GEMM whose tiles would be
// >= 87% padding: the pass reads h once and the (L2-resident) router E x H.
template <int EMAX, int TPW>
__global__ __launch_bounds__(ROUTE_WAVES * 64) void moe_router_route_kernel(
    const half_t* __restrict__ h, int ldh, const half_t* __restrict__ wr, int ldw, int T, int H, int E, int k,
    int norm, int round16, int* __restrict__ ids, float* __restrict__ w) {
  const int lane = threadIdx.x & 63;
  const int t0 = (blockIdx.x * ROUTE_WAVES + (threadIdx.x >> 6)) * TPW;
  if (t0 >= T) return;
  float acc[TPW][EMAX];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
#pragma unroll
    for (int e = 0; e < EMAX; ++e) acc[i][e] = 0.f;
  for (int c = lane * 8; c < H; c += 512) {
    half8 hv[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) hv[i] = *(const half8*)(h + (size_t)min(t0 + i, T - 1) * ldh + c);
#pragma unroll
    for (int e = 0; e < EMAX; ++e) {
      if (e < E) {
        const half8 wv = *(const half8*)(wr + (size_t)e * ldw + c);
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
          for (int r = 0; r < 8; ++r) acc[i][e] = __builtin_fmaf((float)hv[i][r], (float)wv[r], acc[i][e]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    float lg = -INFINITY;
#pragma unroll
    for (int e = 0; e < EMAX; ++e) {
      if (e < E) {
        const float v = warp_sum(acc[i][e]);
        if (lane == e) lg = v;
      }
    }
    if (t0 + i < T) {                                   // wave-uniform
      float l[4] = {lane < E ? (float)(half_t)lg : -INFINITY, -INFINITY, -INFINITY, -INFINITY};
      route_token(l, lane, E, k, norm, round16, (size_t)(t0 + i), ids, w);
    }
  }
}

// Stable counting sort of the n routed entries by expert, in three launches over blocks of
// PB_ENTRIES consecutive entries (entry i = token i / k, slot i % k): per-block histograms, one scan
// block (per-expert offsets, tile prefix, each block's base per expert), then placement: every wave
// keeps its 16 x 64 entries in registers, ranks each 64-entry group by shuffles (rank = earlier
// lanes with the same expert) and advances its per-expert base in LDS.  Entries of an expert keep
// token order, so the plan — and every result computed from it — is deterministic.
constexpr int PB_THREADS = 256;
constexpr int PB_GROUPS = 16;                                  // 64-entry groups per wave
constexpr int PB_ENTRIES = PB_THREADS * PB_GROUPS;            // 4096 entries per block

__global__ __launch_bounds__(PB_THREADS) void moe_hist_kernel(const int* __restrict__ ids, int n, int E,
                                                              int* __restrict__ bhist) {
  __shared__ int hist[MAX_E];
  for (int e = threadIdx.x; e < E; e += PB_THREADS) hist[e] = 0;
  __syncthreads();
  const int base = blockIdx.x * PB_ENTRIES;
  int v[PB_GROUPS];
#pragma unroll
  for (int g = 0; g < PB_GROUPS; ++g) {                        // all loads in flight before the atomics
    const int i = base + g * PB_THREADS + threadIdx.x;
    v[g] = i < n ? ids[i] : -1;
  }
#pragma unroll
  for (int g = 0; g < PB_GROUPS; ++g)
    if (v[g] >= 0) atomicAdd(&hist[v[g]], 1);
  __syncthreads();
  for (int e = threadIdx.x; e < E; e += PB_THREADS) bhist[(size_t)blockIdx.x * E + e] = hist[e];
}

// one block: bhist [B][E] counts -> per-block bases (in place), offs [E+1], tiles [E+1]
__global__ __launch_bounds__(MAX_E) void moe_scan_kernel(int* __restrict__ bhist, int nb, int E,
                                                         int* __restrict__ offs, int* __restrict__ tiles) {
  __shared__ int cnt[MAX_E], off[MAX_E + 1];
  const int e = threadIdx.x;
  if (e < E) {
    int run = 0;
    for (int b = 0; b < nb; ++b) run += bhist[(size_t)b * E + e];
    cnt[e] = run;
  }
  __syncthreads();
  if (e == 0) {
    int o = 0, t = 0;
    offs[0] = 0;
    tiles[0] = 0;
    for (int j = 0; j < E; ++j) {
      off[j] = o;
      o += cnt[j];
      t += (cnt[j] + BM - 1) / BM;
      offs[j + 1] = o;
      tiles[j + 1] = t;
    }
  }
  __syncthreads();
  if (e < E) {
    int run = off[e];
    for (int b = 0; b < nb; ++b) {
      const int c = bhist[(size_t)b * E + e];
      bhist[(size_t)b * E + e] = run;
      run += c;
    }
  }
}

__global__ __launch_bounds__(PB_THREADS) void moe_place_kernel(const int* __restrict__ ids, int n, int k, int E,
                                                               const int* __restrict__ bbase, int* __restrict__ rows,
                                                               int* __restrict__ dest) {
  __shared__ int wbase[PB_THREADS / 64][MAX_E];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < (PB_THREADS / 64) * MAX_E; i += PB_THREADS) (&wbase[0][0])[i] = 0;
  __syncthreads();
  const int wbeg = blockIdx.x * PB_ENTRIES + wave * (64 * PB_GROUPS);
  int v[PB_GROUPS];
#pragma unroll
  for (int g = 0; g < PB_GROUPS; ++g) {
    const int i = wbeg + g * 64 + lane;
    v[g] = i < n ? ids[i] : -1;
  }
#pragma unroll
  for (int g = 0; g < PB_GROUPS; ++g)
    if (v[g] >= 0) atomicAdd(&wbase[wave][v[g]], 1);          // this wave's count per expert
  __syncthreads();
  for (int e = threadIdx.x; e < E; e += PB_THREADS) {        // prefix over the block's waves
    int run = bbase[(size_t)blockIdx.x * E + e];
    for (int w = 0; w < PB_THREADS / 64; ++w) {
      const int c = wbase[w][e];
      wbase[w][e] = run;
      run += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < PB_GROUPS; ++g) {
    const int id = v[g];
    int before = 0, after = 0;
    for (int j = 0; j < 64; ++j) {
      const int o = __shfl(id, j, 64);
      before += (j < lane && o == id) ? 1 : 0;
      after += (j > lane && o == id) ? 1 : 0;
    }
    if (id >= 0) {
      const int i = wbeg + g * 64 + lane;
      const int pos = wbase[wave][id] + before;
      dest[i] = pos;
      rows[pos] = i / k;
    }
    __builtin_amdgcn_wave_barrier();
    if (id >= 0 && after == 0) wbase[wave][id] += before + 1;
    __builtin_amdgcn_wave_barrier();
  }
}

// x[t] = fp16(x[t] + acc), acc = fp16 sum over the token's slots in ascending expert order of
// fp16(y[dest] * w) (+ sh[t], the gated shared-expert output, as one more fp16 add: HF
// Qwen2MoeSparseMoeBlock); one block per token row, 8 columns (16 B) per thread and step
__global__ __launch_bounds__(256) void moe_combine_kernel(const half_t* __restrict__ y, int ldy,
                                                          const int* __restrict__ ids, const int* __restrict__ dest,
                                                          const float* __restrict__ w, half_t* __restrict__ x, int ldx,
                                                          int k, int H, const half_t* __restrict__ sh, int ldsh) {
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
    if (sh) {
      const half8 s = *(const half8*)(sh + (size_t)t * ldsh + c);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = (half_t)((float)acc[q] + (float)s[q]);
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

extern "C" int fls_moe_router_route(const void* h, int ldh, const void* wr, int ldw, int T, int H, int E, int k,
                                    int norm, int round16, int* ids, float* w, fls_stream_t s) {
  if (T <= 0) return 0;
  if (E < 1 || E > 64 || k < 1 || k > MAX_K || k > E || H % 8 || ldh % 8 || ldw % 8) return -2;
  auto hp = (const half_t*)h;
  auto wp = (const half_t*)wr;
  auto st = (hipStream_t)s;
  if (E <= 16) {
    constexpr int TPW = 4;
    hipLaunchKernelGGL((moe_router_route_kernel<16, TPW>), dim3((T + ROUTE_WAVES * TPW - 1) / (ROUTE_WAVES * TPW)),
                       dim3(ROUTE_WAVES * 64), 0, st, hp, ldh, wp, ldw, T, H, E, k, norm, round16, ids, w);
  } else {
    hipLaunchKernelGGL((moe_router_route_kernel<64, 1>), dim3((T + ROUTE_WAVES - 1) / ROUTE_WAVES),
                       dim3(ROUTE_WAVES * 64), 0, st, hp, ldh, wp, ldw, T, H, E, k, norm, round16, ids, w);
  }
  FLS_CHECK_LAUNCH();
  return 0;
}

// bhist: scratch of plan_scratch_ints(n, E) ints
extern "C" int fls_moe_plan_scratch(int n, int E) { return ((n + PB_ENTRIES - 1) / PB_ENTRIES) * E; }

extern "C" int fls_moe_plan(const int* ids, int n, int k, int E, int* offs, int* tiles, int* rows, int* dest,
                            int* bhist, fls_stream_t s) {
  if (E < 1 || E > MAX_E || k < 1 || n < 0) return -2;
  auto st = (hipStream_t)s;
  const int nb = max(1, (n + PB_ENTRIES - 1) / PB_ENTRIES);
  hipLaunchKernelGGL(moe_hist_kernel, dim3(nb), dim3(PB_THREADS), 0, st, ids, n, E, bhist);
  hipLaunchKernelGGL(moe_scan_kernel, dim3(1), dim3(MAX_E), 0, st, bhist, nb, E, offs, tiles);
  hipLaunchKernelGGL(moe_place_kernel, dim3(nb), dim3(PB_THREADS), 0, st, ids, n, k, E, bhist, rows, dest);
  FLS_CHECK_LAUNCH();
  return 0;
}

extern "C" int fls_moe_combine(const void* y, int ldy, const int* ids, const int* dest, const float* w, void* x,
                               int ldx, int T, int k, int H, const void* sh, int ldsh, fls_stream_t s) {
  if (T <= 0) return 0;
  if (k < 1 || k > MAX_K || H % 8 || ldx % 8 || ldy % 8 || (sh && ldsh % 8)) return -2;
  hipLaunchKernelGGL(moe_combine_kernel, dim3(T), dim3(256), 0, (hipStream_t)s, (const half_t*)y, ldy, ids, dest, w,
                     (half_t*)x, ldx, k, H, (const half_t*)sh, ldsh);
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
