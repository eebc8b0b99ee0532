// Memory-bound kernels (gfx950): RMSNorm (optionally row-gathered), token
// embedding gather, vocab softmax, synthetic weight fill, weight dtype casts,
// skinny-M GEMV.
// All loads/stores are 16-byte vectors (guide G13: scalar fp16 loads cost
// ~2x); one 256-thread block per row; fp32 statistics.
#include "common.h"
#include "fls.h"

namespace {

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = warp_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  v = warp_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

// LlamaRMSNorm: y = w * fp16( x * rsqrt(mean(x^2) + eps) )   (HF cast points)
// row r of y <- row (row_idx ? row_idx[r] : r) of x.   H % 8 == 0.
template <int VPT>   // 16-byte vectors per thread held in registers
__global__ __launch_bounds__(256) void rmsnorm_kernel(const half_t* __restrict__ x, const half_t* __restrict__ w,
                                                    half_t* __restrict__ y, const int* __restrict__ row_idx, int H,
                                                    int ldx, int ldy, float eps) {
  __shared__ float red[4];
  const int r = blockIdx.x;
  const int src = row_idx ? row_idx[r] : r;
  const half_t* xr = x + (size_t)src * ldx;
  half_t* yr = y + (size_t)r * ldy;
  const int nvec = H / 8;
  half8 v[VPT];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < nvec) {
      v[i] = *(const half8*)(xr + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += (float)v[i][j] * (float)v[i][j];
    }
  }
  // remainder beyond the register-held part (very large H)
  for (int c = threadIdx.x + VPT * 256; c < nvec; c += 256) {
    const half8 t = *(const half8*)(xr + c * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += (float)t[j] * (float)t[j];
  }
  const float tot = block_sum(ss, red);
  const float inv = rsqrtf(tot / (float)H + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < nvec) {
      const half8 wv = *(const half8*)(w + c * 8);
      half8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (half_t)((float)wv[j] * (float)(half_t)((float)v[i][j] * inv));
      *(half8*)(yr + c * 8) = o;
    }
  }
  for (int c = threadIdx.x + VPT * 256; c < nvec; c += 256) {
    const half8 t = *(const half8*)(xr + c * 8);
    const half8 wv = *(const half8*)(w + c * 8);
    half8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (half_t)((float)wv[j] * (float)(half_t)((float)t[j] * inv));
    *(half8*)(yr + c * 8) = o;
  }
}

// scale != 1: fp16(e * scale) (Granite's embedding_multiplier, GraniteModel's rounding)
__global__ __launch_bounds__(256) void embed_kernel(const int* __restrict__ ids, const half_t* __restrict__ table,
                                                  half_t* __restrict__ out, int H, int V, float scale) {
  const int t = blockIdx.x;
  int id = ids[t];
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);
  const half8* src = (const half8*)(table + (size_t)id * H);
  half8* dst = (half8*)(out + (size_t)t * H);
  if (scale == 1.f) {
    for (int c = threadIdx.x; c < H / 8; c += 256) dst[c] = src[c];
    return;
  }
  for (int c = threadIdx.x; c < H / 8; c += 256) {
    const half8 v = src[c];
    half8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (half_t)((float)v[j] * scale);
    dst[c] = o;
  }
}

// ------------------------------------------------------------ fused RMSNorm pieces
// rstd of one row per wave: the statistic a norm-folded projection applies in its epilogue
// (models/llama.py): the hidden state is read once and nothing is written back but 4 bytes a row.
__global__ __launch_bounds__(256) void row_rstd_kernel(const half_t* __restrict__ x, int ldx,
                                                     const int* __restrict__ row_idx, int rows, int H, float eps,
                                                     float* __restrict__ rstd) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;                            // wave-uniform
  const int lane = threadIdx.x & 63;
  const half_t* xr = x + (size_t)(row_idx ? row_idx[r] : r) * ldx;
  const int nvec = H / 8;
  float ss0 = 0.f, ss1 = 0.f;
  int c = lane;
  for (; c + 64 < nvec; c += 128) {                 // two 16-byte loads in flight per lane
    const half8 a = *(const half8*)(xr + c * 8), b = *(const half8*)(xr + (c + 64) * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ss0 += (float)a[j] * (float)a[j];
      ss1 += (float)b[j] * (float)b[j];
    }
  }
  if (c < nvec) {
    const half8 a = *(const half8*)(xr + c * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss0 += (float)a[j] * (float)a[j];
  }
  const float tot = warp_sum(ss0 + ss1);
  if (lane == 0) rstd[r] = rsqrtf(tot / (float)H + eps);
}

// rstd[r] = rsqrt(sum of the row's partial sums of squares / H + eps): one wave per row, lane j
// holds parts j, j + 64, ... (fixed order), then a fixed butterfly (deterministic)
__global__ __launch_bounds__(256) void rstd_from_ss_kernel(const float* __restrict__ ss, int ss_ld, int nparts,
                                                           int rows, int H, float eps, float* __restrict__ rstd) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;                            // wave-uniform
  const int lane = threadIdx.x & 63;
  float v = 0.f;
  for (int j = lane; j < nparts; j += 64) v += ss[(size_t)r * ss_ld + j];
  v = warp_sum(v);
  if (lane == 0) rstd[r] = rsqrtf(v / (float)H + eps);
}

// W[n, k] *= gamma[k] (fp16 result), 8 columns per thread
__global__ __launch_bounds__(256) void fold_norm_kernel(half_t* __restrict__ w, int ldw, int N, int K,
                                                      const half_t* __restrict__ gamma) {
  const int kv = K / 8;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)N * kv) return;
  const int n = (int)(i / kv), c = (int)(i % kv) * 8;
  half8* p = (half8*)(w + (size_t)n * ldw + c);
  const half8 g = *(const half8*)(gamma + c);
  const half8 v = *p;
  half8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (half_t)((float)v[j] * (float)g[j]);
  *p = o;
}

// y[dst_idx[r]] = x[src_idx[r]] for fp16 rows of H elements (a null index is the identity):
// row gathers / scatters of the pruned last layer and the prefix K/V cache
__global__ __launch_bounds__(256) void copy_rows_kernel(const half_t* __restrict__ x, int ldx,
                                                      const int* __restrict__ src_idx, half_t* __restrict__ y, int ldy,
                                                      const int* __restrict__ dst_idx, int H) {
  const int r = blockIdx.x;
  const half8* src = (const half8*)(x + (size_t)(src_idx ? src_idx[r] : r) * ldx);
  half8* dst = (half8*)(y + (size_t)(dst_idx ? dst_idx[r] : r) * ldy);
  for (int c = threadIdx.x; c < H / 8; c += 256) dst[c] = src[c];
}

// softmax over a row of fp16 logits -> fp16 probabilities (fp32 math),
// online max/sum in one pass, normalisation in a second (row stays in L2).
// inv_scale != 1: the logits are first fp16(l * inv_scale) (Granite's logits / logits_scaling)
__global__ __launch_bounds__(256) void softmax_kernel(const half_t* __restrict__ logits, half_t* __restrict__ probs,
                                                    int V, float inv_scale) {
  const bool scaled = inv_scale != 1.f;
  auto ld = [=](half_t h) { return scaled ? (float)(half_t)((float)h * inv_scale) : (float)h; };
  __shared__ float red[4];
  const half_t* lr = logits + (size_t)blockIdx.x * V;
  half_t* pr = probs + (size_t)blockIdx.x * V;
  float m = -INFINITY, s = 0.f;
  const bool vec = (V % 8) == 0;
  if (vec) {
    for (int c = threadIdx.x; c < V / 8; c += 256) {
      const half8 v = *(const half8*)(lr + c * 8);
      float vm = ld(v[0]);
#pragma unroll
      for (int j = 1; j < 8; ++j) vm = fmaxf(vm, ld(v[j]));
      const float nm = fmaxf(m, vm);
      s *= __expf(m - nm);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf(ld(v[j]) - nm);
      m = nm;
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) {
      const float v = ld(lr[c]);
      const float nm = fmaxf(m, v);
      s = s * __expf(m - nm) + __expf(v - nm);
      m = nm;
    }
  }
  const float gm = block_max(m, red);
  const float gs = block_sum(m == -INFINITY ? 0.f : s * __expf(m - gm), red);
  const float inv = 1.f / gs;
  if (vec) {
    for (int c = threadIdx.x; c < V / 8; c += 256) {
      const half8 v = *(const half8*)(lr + c * 8);
      half8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (half_t)(__expf(ld(v[j]) - gm) * inv);
      *(half8*)(pr + c * 8) = o;
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) pr[c] = (half_t)(__expf(ld(lr[c]) - gm) * inv);
  }
}

// greedy token of each row of fp16 probabilities: the FIRST index of the row's maximum (numpy
// argmax on the scores the reference hands back, main.py:85-88).  Probabilities are >= 0, so
// their bit patterns order like their values; each thread keeps (bits, first index), then a tree
// reduction over the block.
__global__ __launch_bounds__(256) void argmax_rows_kernel(const half_t* __restrict__ x, int ld, int V,
                                                        int* __restrict__ out) {
  __shared__ unsigned sb[256];
  __shared__ int si[256];
  const unsigned short* r = (const unsigned short*)(x + (size_t)blockIdx.x * ld);
  unsigned best = 0;
  int bi = 0x7fffffff;
  for (int c = threadIdx.x; c < V; c += 256) {
    const unsigned b = r[c];
    if (b > best || (b == best && c < bi)) {
      best = b;
      bi = c;
    }
  }
  sb[threadIdx.x] = best;
  si[threadIdx.x] = bi;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      const unsigned b = sb[threadIdx.x + s];
      const int i = si[threadIdx.x + s];
      if (b > sb[threadIdx.x] || (b == sb[threadIdx.x] && i < si[threadIdx.x])) {
        sb[threadIdx.x] = b;
        si[threadIdx.x] = i;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = si[0] == 0x7fffffff ? 0 : si[0];
}

// counter-based normal generator (splitmix64 -> Box-Muller), 8 values/thread
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void fill_random_kernel(half_t* __restrict__ dst, uint64_t n, uint64_t seed,
                                                        float mean, float stdv) {
  const uint64_t base = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (base >= n) return;
  half8 o;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const uint64_t h = splitmix64(seed * 0x2545F4914F6CDD1Dull + base + j);
    const float u1 = ((float)(uint32_t)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
    const float u2 = (float)(uint32_t)(h & 0xFFFFFF) * (1.0f / 16777216.0f);
    const float rr = sqrtf(-2.f * __logf(u1));
    float sn, cs;
    __sincosf(6.28318530718f * u2, &sn, &cs);
    o[j] = (half_t)(mean + stdv * rr * cs);
    o[j + 1] = (half_t)(mean + stdv * rr * sn);
  }
  if (base + 8 <= n) {
    *(half8*)(dst + base) = o;
  } else {
    for (int j = 0; j < 8 && base + j < n; ++j) dst[base + j] = o[j];
  }
}


// ---------------------------------------------------------------- dtype casts
// Weights stream from the checkpoint as raw bytes (runtime/stream.py); bf16 / fp32
// tensors are converted to the fp16 compute dtype on the copy stream once their DMA
// has landed (the reference casts in set_module_tensor_to_device, utils.py:130).
// Round-to-nearest-even, overflow to +-inf: torch's .to(float16).  bf16 -> fp16 may
// run in place (same element size: every thread reads, then rewrites, its own 8
// elements).  8 elements (16 B of output) per thread.
template <int SRC, bool VEC>   // SRC 1 = bf16, 2 = fp32; VEC: 16-byte aligned pointers
__global__ __launch_bounds__(256) void cast_f16_kernel(half_t* dst, const void* src, uint64_t n) {
  const uint64_t base = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (base >= n) return;
  float f[8];
  const int cnt = (VEC && base + 8 <= n) ? 8 : (int)min((uint64_t)8, n - base);
  if constexpr (SRC == 1) {
    const uint16_t* s = (const uint16_t*)src + base;
    if (VEC && cnt == 8) {
      const uint4 v = *(const uint4*)s;
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f[2 * j] = __uint_as_float(w[j] << 16);
        f[2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
      }
    } else {
      for (int j = 0; j < cnt; ++j) f[j] = __uint_as_float((uint32_t)s[j] << 16);
    }
  } else {
    const float* s = (const float*)src + base;
    if (VEC && cnt == 8) {
      const float4 a = *(const float4*)s, b = *(const float4*)(s + 4);
      f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
    } else {
      for (int j = 0; j < cnt; ++j) f[j] = s[j];
    }
  }
  if (VEC && cnt == 8) {
    half8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (half_t)f[j];
    *(half8*)(dst + base) = o;
  } else {
    for (int j = 0; j < cnt; ++j) dst[base + j] = (half_t)f[j];
  }
}

// ---------------------------------------------------------------- skinny GEMV
// C[M, N] = X[M, K] . W[N, K]^T for M <= 16 (LM head of a small batch, K12):
// weight-streaming, one wave per 32 W rows (two v_mfma_f32_16x16x32_f16 tiles
// sharing the X fragment; X rows >= M are zero lanes), four K-steps of loads in
// flight per wave.  W is read exactly once; X (<= 256 KB) stays in L2.
constexpr int GV_U = 4;
__global__ __launch_bounds__(256) void gemv_skinny_kernel(const half_t* __restrict__ X, const half_t* __restrict__ W,
                                                          half_t* __restrict__ C, int M, int N, int K, int ldx,
                                                          int ldw, int ldc) {
  const int lane = threadIdx.x & 63;
  const int n0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 32;
  if (n0 >= N) return;
  const int fr = lane & 15, grp = lane >> 4;
  const half_t* wa = W + (size_t)min(n0 + fr, N - 1) * ldw + grp * 8;
  const half_t* wb = W + (size_t)min(n0 + 16 + fr, N - 1) * ldw + grp * 8;
  const bool xrow = fr < M;
  const half_t* xp = X + (size_t)(xrow ? fr : 0) * ldx + grp * 8;
  floatx4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
  const half8 zero = {};
  int k = 0;
  for (; k + 32 * GV_U <= K; k += 32 * GV_U) {
    half8 fa[GV_U], fb[GV_U], fx[GV_U];
#pragma unroll
    for (int u = 0; u < GV_U; ++u) {
      fa[u] = __builtin_nontemporal_load((const half8*)(wa + k + u * 32));
      fb[u] = __builtin_nontemporal_load((const half8*)(wb + k + u * 32));
      fx[u] = xrow ? *(const half8*)(xp + k + u * 32) : zero;
    }
#pragma unroll
    for (int u = 0; u < GV_U; ++u) {
      a0 = mfma16x16x32(fa[u], fx[u], a0);
      a1 = mfma16x16x32(fb[u], fx[u], a1);
    }
  }
  for (; k < K; k += 32) {
    const half8 fa = *(const half8*)(wa + k), fb = *(const half8*)(wb + k);
    const half8 fx = xrow ? *(const half8*)(xp + k) : zero;
    a0 = mfma16x16x32(fa, fx, a0);
    a1 = mfma16x16x32(fb, fx, a1);
  }
  // lane holds D[n = 4*grp + r][m = fr] of each 16x16 tile
  if (!xrow) return;
  half_t* cp = C + (size_t)fr * ldc;
  const int na = n0 + 4 * grp, nb = n0 + 16 + 4 * grp;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (na + r < N) cp[na + r] = (half_t)a0[r];
    if (nb + r < N) cp[nb + r] = (half_t)a1[r];
  }
}
// Qwen3 q/k head norm + RoPE, in place on the projection output:
//   head h < n_q:        x_h <- rope( fp16( qn * fp16( x_h * rsqrt(mean(x_h^2) + eps) ) ) )
//   n_q <= h < n_q+n_k:  same with kn
// (HF Qwen3RMSNorm cast points, then rotate-half RoPE in fp32 on the normalised fp16 values).
// One wave per (row, head): lane p holds the rotate-half pair (p, p + hd/2), so the norm is one
// wave reduction and the rotation lane-local.  hd in {64, 96, 128}.  qn == nullptr: RoPE only (the
// unfused path for head sizes the GEMM's RoPE epilogue does not tile: Phi-3-mini's 96).
__global__ __launch_bounds__(256) void headnorm_rope_kernel(half_t* __restrict__ x, int ldx, int rows, int n_q,
                                                          int n_k, const half_t* __restrict__ qn,
                                                          const half_t* __restrict__ kn, const int* __restrict__ pos,
                                                          const float* __restrict__ cos_t,
                                                          const float* __restrict__ sin_t, int hd, float eps) {
  const int r = blockIdx.x;
  const int h = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int p = threadIdx.x & 63;
  const int half = hd >> 1;
  if (r >= rows || h >= n_q + n_k) return;          // wave-uniform
  half_t* xh = x + (size_t)r * ldx + (size_t)h * hd;
  const half_t* w = h < n_q ? qn : kn;
  const bool on = p < half;
  const float a = on ? (float)xh[p] : 0.f;
  const float b = on ? (float)xh[p + half] : 0.f;
  float na = a, nb = b;
  if (qn != nullptr) {                              // kernel-uniform
    const float ss = warp_sum(a * a + b * b);
    const float rs = rsqrtf(ss / (float)hd + eps);
    na = (float)(half_t)((float)w[p] * (float)(half_t)(a * rs));
    nb = (float)(half_t)((float)w[p + half] * (float)(half_t)(b * rs));
  }
  if (!on) return;
  const int q = pos[r];
  const float c = cos_t[(size_t)q * half + p], sn = sin_t[(size_t)q * half + p];
  xh[p] = (half_t)(na * c - nb * sn);
  xh[p + half] = (half_t)(nb * c + na * sn);
}

}  // namespace

extern "C" int fls_headnorm_rope(void* x, int ldx, int rows, int n_q, int n_k, const void* qn, const void* kn,
                                 const int* pos, const float* cos_t, const float* sin_t, int hd, float eps,
                                 fls_stream_t s) {
  if (rows <= 0 || n_q + n_k <= 0) return 0;
  if (hd != 64 && hd != 96 && hd != 128) return -3;
  if ((qn == nullptr) != (kn == nullptr)) return -2;
  dim3 grid(rows, (n_q + n_k + 3) / 4);
  hipLaunchKernelGGL(headnorm_rope_kernel, grid, dim3(256), 0, (hipStream_t)s, (half_t*)x, ldx, rows, n_q, n_k,
                     (const half_t*)qn, (const half_t*)kn, pos, cos_t, sin_t, hd, eps);
  FLS_CHECK_LAUNCH();
  return 0;
}

extern "C" int fls_rmsnorm(const void* x, const void* w, void* y, const int* row_idx, int rows, int H, int ldx,
                           int ldy, float eps, fls_stream_t s) {
  if (rows <= 0) return 0;
  if (H % 8 || ldx % 8 || ldy % 8) return -2;
  auto st = (hipStream_t)s;
  const int nvec = H / 8;
  if (nvec <= 256)
    hipLaunchKernelGGL(rmsnorm_kernel<1>, dim3(rows), dim3(256), 0, st, (const half_t*)x, (const half_t*)w,
                       (half_t*)y, row_idx, H, ldx, ldy, eps);
  else if (nvec <= 512)
    hipLaunchKernelGGL(rmsnorm_kernel<2>, dim3(rows), dim3(256), 0, st, (const half_t*)x, (const half_t*)w,
                       (half_t*)y, row_idx, H, ldx, ldy, eps);
  else
    hipLaunchKernelGGL(rmsnorm_kernel<4>, dim3(rows), dim3(256), 0, st, (const half_t*)x, (const half_t*)w,
                       (half_t*)y, row_idx, H, ldx, ldy, eps);
  FLS_CHECK_LAUNCH();
  return 0;
}

extern "C" int fls_embed(const int* ids, const void* table, void* out, int T, int H, int V, float scale,
                         fls_stream_t s) {
  if (T <= 0) return 0;
  if (H % 8) return -2;
  hipLaunchKernelGGL(embed_kernel, dim3(T), dim3(256), 0, (hipStream_t)s, ids, (const half_t*)table, (half_t*)out,
                     H, V, scale);
  FLS_CHECK_LAUNCH();
  return 0;
}

extern "C" int fls_softmax_rows(const void* logits, void* probs, int rows, int V, float inv_scale, fls_stream_t s) {
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(softmax_kernel, dim3(rows), dim3(256), 0, (hipStream_t)s, (const half_t*)logits,
                     (half_t*)probs, V, inv_scale);
  FLS_CHECK_LAUNCH();
  return 0;
}

extern "C" int fls_argmax_rows(const void* x, int ld, int rows, int V, int* out, fls_stream_t s) {
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(argmax_rows_kernel, dim3(rows), dim3(256), 0, (hipStream_t)s, (const half_t*)x, ld, V, out);
  FLS_CHECK_LAUNCH();
  return 0;
}

extern "C" int fls_row_rstd(const void* x, int ldx, const int* row_idx, int rows, int H, float eps, float* rstd,
                            fls_stream_t s) {
  if (rows <= 0) return 0;
  if (H % 8 || ldx % 8 || ((uintptr_t)x & 15)) return -2;
  hipLaunchKernelGGL(row_rstd_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)s, (const half_t*)x, ldx,
                     row_idx, rows, H, eps, rstd);
  FLS_CHECK_LAUNCH();
  return 0;
}

extern "C" int fls_rstd_from_ss(const float* ss, int ss_ld, int nparts, int rows, int H, float eps, float* rstd,
                                fls_stream_t s) {
  if (rows <= 0) return 0;
  if (nparts <= 0 || ss_ld < nparts) return -2;
  hipLaunchKernelGGL(rstd_from_ss_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)s, ss, ss_ld, nparts, rows,
                     H, eps, rstd);
  FLS_CHECK_LAUNCH();
  return 0;
}

extern "C" int fls_fold_norm(void* w, int ldw, int N, int K, const void* gamma, fls_stream_t s) {
  if (N <= 0 || K <= 0) return 0;
  if (K % 8 || ldw % 8 || (((uintptr_t)w | (uintptr_t)gamma) & 15)) return -2;
  const long long threads = (long long)N * (K / 8);
  hipLaunchKernelGGL(fold_norm_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)s,
                     (half_t*)w, ldw, N, K, (const half_t*)gamma);
  FLS_CHECK_LAUNCH();
  return 0;
}

// grid-stride 16-byte copy on a fixed number of workgroups (an RCCL-like channel count)
__global__ __launch_bounds__(256) void copy_blocks_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                        size_t n16) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

// device-to-device copy of `bytes` (16-byte multiple): mode 0 the HIP runtime's copy (a blit kernel on
// the CUs), 1 hipMemcpyDeviceToDeviceNoCU (the SDMA engines, no compute unit), 2 copy_blocks_kernel on
// `blocks` workgroups.  bench.py --emulate-dp-fanout: the data-parallel weight all-gather's HBM traffic
// on one GPU, on the CUs or off them
extern "C" int fls_copy_d2d(void* dst, const void* src, uint64_t bytes, int mode, int blocks, fls_stream_t s) {
  if (!bytes) return 0;
  if (bytes % 16) return -2;
  if (mode == 2) {
    hipLaunchKernelGGL(copy_blocks_kernel, dim3(blocks > 0 ? blocks : 32), dim3(256), 0, (hipStream_t)s,
                       (const uint4*)src, (uint4*)dst, (size_t)(bytes / 16));
    FLS_CHECK_LAUNCH();
    return 0;
  }
  return hipMemcpyAsync(dst, src, bytes, mode == 1 ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToDevice,
                        (hipStream_t)s) == hipSuccess ? 0 : -1;
}

extern "C" int fls_copy_rows(const void* x, int ldx, const int* src_idx, void* y, int ldy, const int* dst_idx,
                             int rows, int H, fls_stream_t s) {
  if (rows <= 0) return 0;
  if (H % 8 || ldx % 8 || ldy % 8 || (((uintptr_t)x | (uintptr_t)y) & 15)) return -2;
  hipLaunchKernelGGL(copy_rows_kernel, dim3(rows), dim3(256), 0, (hipStream_t)s, (const half_t*)x, ldx, src_idx,
                     (half_t*)y, ldy, dst_idx, H);
  FLS_CHECK_LAUNCH();
  return 0;
}

extern "C" int fls_fill_random(void* dst, uint64_t n_elems, uint64_t seed, float mean, float stdv, fls_stream_t s) {
  if (n_elems == 0) return 0;
  const uint64_t threads = (n_elems + 7) / 8;
  const uint64_t blocks = (threads + 255) / 256;
  hipLaunchKernelGGL(fill_random_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)s, (half_t*)dst, n_elems,
                     seed, mean, stdv);
  FLS_CHECK_LAUNCH();
  return 0;
}

// dst[i] = fp16(src[i]) for src_dtype 1 = bf16 (dst may equal src), 2 = fp32 (no overlap)
extern "C" int fls_cast_f16(void* dst, const void* src, int src_dtype, uint64_t n, fls_stream_t s) {
  if (n == 0) return 0;
  if (src_dtype == 2 && (const char*)dst < (const char*)src + 4 * n && (const char*)src < (const char*)dst + 2 * n)
    return -3;
  if (src_dtype == 1 && dst != src && (const char*)dst < (const char*)src + 2 * n &&
      (const char*)src < (const char*)dst + 2 * n)
    return -3;
  const bool vec = ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0);
  const uint64_t blocks = ((n + 7) / 8 + 255) / 256;
  auto st = (hipStream_t)s;
  const dim3 g((unsigned)blocks), b(256);
  if (src_dtype == 1 && vec) hipLaunchKernelGGL((cast_f16_kernel<1, true>), g, b, 0, st, (half_t*)dst, src, n);
  else if (src_dtype == 1) hipLaunchKernelGGL((cast_f16_kernel<1, false>), g, b, 0, st, (half_t*)dst, src, n);
  else if (src_dtype == 2 && vec) hipLaunchKernelGGL((cast_f16_kernel<2, true>), g, b, 0, st, (half_t*)dst, src, n);
  else if (src_dtype == 2) hipLaunchKernelGGL((cast_f16_kernel<2, false>), g, b, 0, st, (half_t*)dst, src, n);
  else return -1;
  FLS_CHECK_LAUNCH();
  return 0;
}

extern "C" int fls_gemv_skinny(const void* x, const void* w, void* c, int M, int N, int K, int ldx, int ldw, int ldc,
                               fls_stream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 16 || K % 32 || ldx % 8 || ldw % 8) return -2;
  const int waves = (N + 31) / 32;
  hipLaunchKernelGGL(gemv_skinny_kernel, dim3((waves + 3) / 4), dim3(256), 0, (hipStream_t)s, (const half_t*)x,
                     (const half_t*)w, (half_t*)c, M, N, K, ldx, ldw, ldc);
  FLS_CHECK_LAUNCH();
  return 0;
}
