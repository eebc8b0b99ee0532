// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 half_t;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((vector_size(8)));

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

constexpr int WAVE = 64;

__device__ __forceinline__ floatx4 mfma16x16x32(half8 a, half8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// In-place accumulate on an AGPR-resident accumulator (dst tied to srcC), also a compiler
// memory barrier: LDS reads / LDS-DMA written between these statements issue exactly in
// source order (hand-interleaved schedules).  Used where all 256 AGPRs hold accumulators: the
// builtin lets the register allocator rename dst != srcC, which with zero spare AGPRs turns
// into copies and spills.  The caller owns MFMA->VALU hazards on `c` after the last use.
__device__ __forceinline__ void mfma_acc_inplace_ordered(floatx4& c, const half8& a, const half8& b) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b) : "memory");
}

// 16-byte global -> LDS DMA (dest = wave-uniform base + lane*16)
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const GLB_AS void*)gsrc, (LDS_AS void*)lds_wave_base, 16, 0, 0);
}

// transposed LDS read: 4 rows x 16 cols block per 16-lane group (T10)
__device__ __forceinline__ half4 ds_read_tr16(const void* lds_addr) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)lds_addr);
  return __builtin_bit_cast(half4, v);
}

__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }

#define FLS_CHECK_LAUNCH()                                  \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return (int)_e;                   \
  } while (0)
