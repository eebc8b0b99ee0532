// Shared pieces of the MFMA projection GEMMs (gfx950): epilogues, tile order and the v10
// 256x256x64 kernel.  Included by gemm.hip (dense projections) and moe.hip (grouped expert
// GEMMs) -- each translation unit instantiates only its own variants, so adding the grouped
// kernels does not perturb the dense kernels' code generation (guide §5.4 rule 19).
#pragma once
#include "common.h"
#include "fls.h"

#include <cstdlib>
#include <type_traits>

namespace {


constexpr int BM = 256, BN = 256, BK = 64;
// internal epilogue code: RoPE with head_dim 64 (FLS_EPI_ROPE inside this file means head_dim 128);
// a compile-time head dim keeps the v10 RoPE epilogue free of spills
constexpr int EPI_ROPE64 = 4;
// internal: split-K partial — raw fp32 accumulators of a K slice to a [S][M][N] workspace (the
// epilogue runs in splitk_reduce_kernel, gemm.hip)
constexpr int EPI_F32 = 6;
constexpr bool is_rope(int epi) { return epi == FLS_EPI_ROPE || epi == EPI_ROPE64; }
constexpr int BUF = 65536;    // one K-tile stage: X image (32 KiB) then W image (32 KiB)
constexpr int WIMG = 32768;

struct Epi {
  const half_t* R;
  int ldr;
  const int* pos;
  const float* cos_t;
  const float* sin_t;
  int rope_cols;
  int head_dim;
  const half_t* bias;   // optional per-output-column bias (Qwen2 q/k/v, Llama attention_bias), added first
  int gu_rows;          // SWIGLU: I (rows of gate = rows of up)
  int order;            // v10 tile order (tile_of), set by the launcher
  // grouped v10 (mixture-of-experts; moe.hip): see gemm_nt_v10<EPI, true>
  const int* g_tiles;
  const int* g_offs;
  const int* g_rows;
  long long g_wstride;
  int g_n;
  // split-K (EPI_F32): K slices per tile, elements per slice, fp32 workspace elements per slice
  int ksplit;
  int kslice;
  long long part_stride;
  // optional per-row scale of the raw product (fp32 [M], row m of A): the RMSNorm statistic
  // rsqrt(mean(x^2) + eps) of a GEMM that reads the un-normalised hidden state x with the norm
  // weight folded into W (fused RMSNorm + projection); applied before the bias
  const float* rs = nullptr;
  // scale of (product + bias) before the residual add (Granite's residual_multiplier)
  float alpha = 1.f;
  // optional (RESID): per-row partial sums of squares of the fp16 output, one fp32 per 128 output
  // columns: ss[m * ss_ld + n / 128].  The next fused-norm GEMM's row statistic is their sum
  // (fls_rstd_from_ss) -- the separate pass over the hidden state (row_rstd) is not needed
  float* ss = nullptr;
  int ss_ld = 0;
  // FLS_GEMM_ROW_EXACT: only the row-independent paths (v10 / v11 / mid-M tiles, or the generic kernel
  // for shapes they do not take): every output row gets the same arithmetic whatever M and the other rows
  int row_exact = 0;
};

// sum of v over the 4 lanes of one output row (lanes l, l^16, l^32, l^48: one 16-column group
// each); every lane gets the same value, in a fixed order (deterministic).  All lanes must run it.
__device__ __forceinline__ float row_sum_4groups(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// one lane's share of a row's partial sum of squares over a pair of 16-column subtiles (its 4 columns
// of each), in one fixed order of explicit FMAs: the v10 / v11 residual epilogue and ss_partials_kernel
// (every other GEMM path, and the fused norm's statistic of a hidden state no residual GEMM left
// partials for) run this same code on the same lane layout, so their partials are bitwise equal
__device__ __forceinline__ float ss_accum_pair(float sq, const half4& oa, const half4& ob) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float a = (float)oa[r], b = (float)ob[r];
    sq = __builtin_fmaf(a, a, sq);
    sq = __builtin_fmaf(b, b, sq);
  }
  return sq;
}

// the per-row scale of row m (1 without one: x * 1.0f is exact, so the unscaled path is unchanged)
__device__ __forceinline__ float row_scale(const Epi& ep, int m) { return ep.rs ? ep.rs[m] : 1.f; }

// SWIGLU logical row l (gate/up interleaved per 16 rows) -> physical row of [gate; up]
__device__ __forceinline__ int gu_phys_row(int l, int I) {
  return ((l >> 4) & 1) * I + (l >> 5) * 16 + (l & 15);
}

// Store one pair of neighbouring 16-column subtiles (cols n_first + off + r and +16) of row m.
template <int EPI>
__device__ __forceinline__ void store_pair_off(half_t* __restrict__ C, int ldc, int m, int n_first, int off,
                                               const floatx4& acc_a, const floatx4& acc_b, const Epi& ep) {
  const int c0 = n_first + off;
  if constexpr (EPI == FLS_EPI_SWIGLU) {
    // pair = (gate, up) of intermediate columns [n_first/2, n_first/2 + 16)
    const int oc = n_first / 2 + off;
    const float s = row_scale(ep, m);
    half4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (half_t)(silu(acc_a[r] * s) * (acc_b[r] * s));
    *(half4*)(C + (size_t)m * ldc + oc) = o;
    return;
  } else {
    const float s = row_scale(ep, m);
    floatx4 a = acc_a * s, b = acc_b * s;
    if (ep.bias) {
      const half4 ba = *(const half4*)(ep.bias + c0);
      const half4 bb = *(const half4*)(ep.bias + c0 + 16);
#pragma unroll
      for (int r = 0; r < 4; ++r) { a[r] += (float)ba[r]; b[r] += (float)bb[r]; }
    }
    if constexpr (EPI == FLS_EPI_RESID) {
      const half4 ra = *(const half4*)(ep.R + (size_t)m * ep.ldr + c0);
      const half4 rb = *(const half4*)(ep.R + (size_t)m * ep.ldr + c0 + 16);
#pragma unroll
      for (int r = 0; r < 4; ++r) { a[r] = a[r] * ep.alpha + (float)ra[r]; b[r] = b[r] * ep.alpha + (float)rb[r]; }
    }
    half4 oa, ob;
#pragma unroll
    for (int r = 0; r < 4; ++r) { oa[r] = (half_t)a[r]; ob[r] = (half_t)b[r]; }
    *(half4*)(C + (size_t)m * ldc + c0) = oa;
    *(half4*)(C + (size_t)m * ldc + c0 + 16) = ob;
  }
}

// RoPE pair: columns ca (first half of a head) and ca + hd/2 of row m; f = ca % hd.  The arithmetic
// is epilogue_rope's, expression for expression (x = acc * s + bias, then the rotation), so the mid-M
// kernel's rows are bitwise the v10 / v11 rows (row-exact calls take either)
__device__ __forceinline__ void store_rope_pair(half_t* __restrict__ C, int ldc, int m, int ca, const floatx4& acc_a,
                                                const floatx4& acc_b, const Epi& ep) {
  const int hd = ep.head_dim, half_hd = hd >> 1;
  const int cb = ca + half_hd;
  const float s = row_scale(ep, m);
  half4 ba = half4{0, 0, 0, 0}, bb = half4{0, 0, 0, 0};
  if (ep.bias) {
    ba = *(const half4*)(ep.bias + ca);
    bb = *(const half4*)(ep.bias + cb);
  }
  const bool rot = ca < ep.rope_cols;
  floatx4 cs, sn;
  if (rot) {
    const int p = ep.pos[m];
    cs = *(const floatx4*)(ep.cos_t + (size_t)p * half_hd + (ca % hd));
    sn = *(const floatx4*)(ep.sin_t + (size_t)p * half_hd + (ca % hd));
  }
  half4 oa, ob;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float x1 = __builtin_fmaf(acc_a[r], s, (float)ba[r]), x2 = __builtin_fmaf(acc_b[r], s, (float)bb[r]);
    if (rot) {
      const float c = cs[r], sv = sn[r];
      const float y1 = __builtin_fmaf(x1, c, -(x2 * sv)), y2 = __builtin_fmaf(x2, c, x1 * sv);
      x1 = y1;
      x2 = y2;
    }
    oa[r] = (half_t)x1;
    ob[r] = (half_t)x2;
  }
  *(half4*)(C + (size_t)m * ldc + ca) = oa;
  *(half4*)(C + (size_t)m * ldc + cb) = ob;
}

// 16-byte stores of a pair of neighbouring 16-column subtiles (columns c .. c+31 of one row).
// Lanes of row group g (lane >> 4) hold columns 4g..4g+3 of both subtiles; one v_permlane16_swap
// per dword exchanges the odd groups' first-subtile halves with the even groups' second-subtile
// halves, after which every lane owns 8 consecutive columns: g0 -> c+0, g2 -> c+8, g1 -> c+16,
// g3 -> c+24.  Half the store instructions, and each 16-lane group writes whole 64-B segments.
// Every lane must execute the swap (partners share the row, so a row guard belongs on the store).
__device__ __forceinline__ uint4 wide_pair(half4 oa, half4 ob) {
  const uint2 a = __builtin_bit_cast(uint2, oa), b = __builtin_bit_cast(uint2, ob);
  const auto r0 = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  return uint4{r0[0], r1[0], r0[1], r1[1]};
}
__device__ __forceinline__ int wide_off(int g) { return (g & 1) * 16 + (g >> 1) * 8; }

// Inverse of wide_pair on a 16-byte row chunk loaded at wide_off (the swap is an involution):
// returns this lane's 4 columns of the first and of the second subtile.
__device__ __forceinline__ void unwide_pair(uint4 v, half4& a, half4& b) {
  const auto r0 = __builtin_amdgcn_permlane16_swap(v.x, v.z, false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(v.y, v.w, false, false);
  a = __builtin_bit_cast(half4, uint2{r0[0], r1[0]});
  b = __builtin_bit_cast(half4, uint2{r0[1], r1[1]});
}

// RoPE epilogue of a v10 wave quadrant (128 rows x 128 columns = whole heads).
// HD 128: one head per wave, pairs (q, q+4); HD 64: two heads, pairs (q', q'+2),
// q' in {0, 1, 4, 5}.  Neighbouring subtiles (q, q+1), q even, leave as 16-byte stores
// (wide_pair).  Row group u+1's cos/sin loads are issued before row group u's stores (the
// tables cannot alias C, so a fence keeps the compiler from hoisting all 8 rows' loads and
// spilling).
template <int HD, int U = 8, bool LO = false>
__device__ __forceinline__ void epilogue_rope(half_t* __restrict__ C, int ldc, int M, int mrow0, int ncol0, int grp,
                                              floatx4 (&acc)[U][8], const Epi& ep, int mlo = 0) {
  constexpr int HS = HD / 32;
  constexpr int HALF = HD / 2;
  const int off = 4 * grp;
  const int woff = wide_off(grp);
  int pos[U];
#pragma unroll
  for (int u = 0; u < U; ++u) pos[u] = ep.pos[min(mrow0 + u * 16, M - 1)];
  const float* const rsp = ep.rs;
  int f0[4];
  bool rot[4];
  half4 ba[4], bb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int ta = HD == 128 ? q : (q & 1) + (q >> 1) * 4;
    const int ca = ncol0 + ta * 16;
    f0[q] = (ta * 16) % HD + off;
    rot[q] = ca < ep.rope_cols;                      // wave-uniform
    if (ep.bias) {
      ba[q] = *(const half4*)(ep.bias + ca + off);
      bb[q] = *(const half4*)(ep.bias + ca + HALF + off);
    } else {
      ba[q] = half4{0, 0, 0, 0};
      bb[q] = half4{0, 0, 0, 0};
    }
  }
  floatx4 cs[2][4], sn[2][4];
  auto load = [&](int u, int sl) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (rot[q]) {
        cs[sl][q] = *(const floatx4*)(ep.cos_t + (size_t)pos[u] * HALF + f0[q]);
        sn[sl][q] = *(const floatx4*)(ep.sin_t + (size_t)pos[u] * HALF + f0[q]);
      }
    }
  };
  load(0, 0);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int sl = u & 1;
    if (u + 1 < U) load(u + 1, sl ^ 1);
    asm volatile("" ::: "memory");
    const int m = mrow0 + u * 16;
    const float s = rsp ? rsp[min(m, M - 1)] : 1.f;
    half4 oa[4], ob[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ta = HD == 128 ? q : (q & 1) + (q >> 1) * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // explicit fmas: every kernel with a RoPE epilogue rounds the same way (store_rope_pair)
        float x1 = __builtin_fmaf(acc[u][ta][r], s, (float)ba[q][r]);
        float x2 = __builtin_fmaf(acc[u][ta + HS][r], s, (float)bb[q][r]);
        if (rot[q]) {
          const float c = cs[sl][q][r], sv = sn[sl][q][r];
          const float y1 = __builtin_fmaf(x1, c, -(x2 * sv)), y2 = __builtin_fmaf(x2, c, x1 * sv);
          x1 = y1;
          x2 = y2;
        }
        oa[q][r] = (half_t)x1;
        ob[q][r] = (half_t)x2;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; q += 2) {
      const int ta = HD == 128 ? q : (q & 1) + (q >> 1) * 4;
      const uint4 va = wide_pair(oa[q], oa[q + 1]);
      const uint4 vb = wide_pair(ob[q], ob[q + 1]);
      half_t* cp = C + (size_t)m * ldc + ncol0 + ta * 16 + woff;
      if (m < M && (!LO || m >= mlo)) {
        *(uint4*)cp = va;
        *(uint4*)(cp + HALF) = vb;
      }
    }
  }
}

// Epilogue of a wave's 128 (M) x 128 (N) quadrant held as acc[8 row groups][8 subtiles] (v10),
// 16-byte stores throughout (wide_pair).  Row group u+1's operand loads (residual rows) are issued
// before row group u's stores (different rows, so in-place R == C stays correct); the per-column
// bias is loaded once.
// U row groups (v10: 8; v11: 12).  LO: the block stores only rows >= mlo (v11's last M tile is
// shifted back to end at row M, so it recomputes rows its neighbour owns; storing them twice
// would be wrong for the in-place residual).
template <int EPI, int U = 8, bool LO = false>
__device__ __forceinline__ void epilogue_quadrant(half_t* __restrict__ C, int ldc, int M, int mrow0, int ncol0,
                                                  int grp, floatx4 (&acc)[U][8], const Epi& ep, int mlo = 0) {
  if constexpr (EPI == EPI_F32) {                    // split-K partial: fp32, ldc in floats
    float* Cf = (float*)C;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = mrow0 + u * 16;
      if (m < M && (!LO || m >= mlo)) {
#pragma unroll
        for (int t = 0; t < 8; ++t) *(floatx4*)(Cf + (size_t)m * ldc + ncol0 + t * 16 + 4 * grp) = acc[u][t];
      }
    }
    return;
  } else if constexpr (EPI == FLS_EPI_ROPE) {
    epilogue_rope<128, U, LO>(C, ldc, M, mrow0, ncol0, grp, acc, ep, mlo);
    return;
  } else if constexpr (EPI == EPI_ROPE64) {
    epilogue_rope<64, U, LO>(C, ldc, M, mrow0, ncol0, grp, acc, ep, mlo);
    return;
  } else {
    const int off = 4 * grp;
    const int woff = wide_off(grp);
    if constexpr (EPI == FLS_EPI_SWIGLU) {
      // pair p -> intermediate columns [ncol0/2 + 16p, +16); pairs (p, p+1) share one 16-B store
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int m = mrow0 + u * 16;
        const float s = ep.rs ? ep.rs[min(m, M - 1)] : 1.f;
        half4 o[4];
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[p][r] = (half_t)(silu(acc[u][2 * p][r] * s) * (acc[u][2 * p + 1][r] * s));
#pragma unroll
        for (int p = 0; p < 4; p += 2) {
          const uint4 v = wide_pair(o[p], o[p + 1]);
          if (m < M && (!LO || m >= mlo)) *(uint4*)(C + (size_t)m * ldc + ncol0 / 2 + p * 16 + woff) = v;
        }
      }
      return;
    } else {
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
      uint4 rw[2][4];
      auto load = [&](int u, int sl) {
        if constexpr (EPI == FLS_EPI_RESID) {
          const int m = min(mrow0 + u * 16, M - 1);
          const half_t* rp = ep.R + (size_t)m * ep.ldr + ncol0 + woff;
#pragma unroll
          for (int p = 0; p < 4; ++p) rw[sl][p] = *(const uint4*)(rp + p * 32);
        }
      };
      // RESID with ep.ss: this wave's 128 columns of each row -> one partial sum of squares
      float* const ssp = EPI == FLS_EPI_RESID ? ep.ss : nullptr;
      auto body = [&](auto has_bias) {
        load(0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int sl = u & 1;
          if (u + 1 < U) load(u + 1, sl ^ 1);
          asm volatile("" ::: "memory");
          const int m = mrow0 + u * 16;
          const float s = ep.rs ? ep.rs[min(m, M - 1)] : 1.f;
          float sq = 0.f;
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            floatx4 a = acc[u][2 * p] * s, b = acc[u][2 * p + 1] * s;
            if constexpr (decltype(has_bias)::value) {
#pragma unroll
              for (int r = 0; r < 4; ++r) { a[r] += (float)ba[p][r]; b[r] += (float)bb[p][r]; }
            }
            if constexpr (EPI == FLS_EPI_RESID) {
              half4 ra, rb;
              unwide_pair(rw[sl][p], ra, rb);
#pragma unroll
              for (int r = 0; r < 4; ++r) { a[r] = a[r] * ep.alpha + (float)ra[r]; b[r] = b[r] * ep.alpha + (float)rb[r]; }
            }
            half4 oa, ob;
#pragma unroll
            for (int r = 0; r < 4; ++r) { oa[r] = (half_t)a[r]; ob[r] = (half_t)b[r]; }
            if constexpr (EPI == FLS_EPI_RESID) {
              if (ssp) sq = ss_accum_pair(sq, oa, ob);
            }
            const uint4 v = wide_pair(oa, ob);
            if (m < M && (!LO || m >= mlo)) *(uint4*)(C + (size_t)m * ldc + ncol0 + p * 32 + woff) = v;
          }
          if constexpr (EPI == FLS_EPI_RESID) {
            if (ssp) {                                 // wave-uniform
              sq = row_sum_4groups(sq);
              if (grp == 0 && m < M && (!LO || m >= mlo)) ssp[(size_t)m * ep.ss_ld + (ncol0 >> 7)] = sq;
            }
          }
        }
      };
      if (ep.bias) body(std::true_type{});
      else body(std::false_type{});
    }
  }
}

// Columns of the 4 accumulator subtiles of a wave that owns 64 columns of a 128-column group
// (mid / generic kernels).  RoPE with hd 128 splits the group so that both halves of every
// head pair stay in one wave: subtiles (0, 2) and (1, 3) are rotation partners.
__device__ __forceinline__ int sub_col(bool rope128, int wn, int t) {
  return rope128 ? (t >> 1) * 64 + wn * 32 + (t & 1) * 16 : wn * 64 + t * 16;
}

// ------------------------------------------------------------------ v10
// 256x256x64 tile, 4 waves = one per SIMD, 128x128 outputs per wave in 256 AGPR
// accumulators (2/3 of the LDS fragment reads per FLOP of an 8-wave 256x256 kernel).
// The register read-ahead is one phase deep (registers are private, they need no
// barrier); the shared-LDS hazards are synchronised once per super-phase (SP = two
// phases of 32 MFMAs = one 64x64 quadrant x K=64 each):
//   SP0 of tile t: DMA XA(t+2) + W-first(t+2)    SP1 of tile t: DMA W-second(t+2) + XB(t+2)
// (tile t's data is read in SPs 2t-1 and 2t, so each region is refilled in the SP after
// its last reads, and every half-tile is read 3 SPs after issue: `vmcnt(16)` = 2 SPs x
// 2 half-tiles x 4 ops stay in flight at each barrier).  Per phase: 32 MFMAs with one
// ds_read_b128 after each of the first 16 even-numbered MFMAs (the 8 reads of the half
// needed later) and the half-tile's 4 LDS-DMA ops after MFMAs 17, 20, 23, 26; then
// lgkmcnt(0) + counted vmcnt + raw barrier.  Requires an even number of K-tiles.
//
// W-operand source addresses are per 8-row piece, so the SWIGLU loader can map the
// logical (gate/up interleaved) tile rows onto the stacked [gate; up] weight.

// Virtual tile id -> (tm, tn).  order > 0: groups of `order` M tiles walked M-fastest along N;
// order < 0: groups of -order N tiles walked N-fastest along M.  With the XCD-aware remap
// (virtual ids [x*q, (x+1)*q) run on XCD x) a group of tiles/8 makes each XCD own one chunk of
// the grouped dimension's operand, which stays in its L2 / the MALL, while all XCDs walk the
// other operand in step (profiles/r2_gemm).
__device__ __forceinline__ int2 tile_of(int b, int tiles_m, int tiles_n, int order) {
  const bool by_m = order > 0;
  const int g = by_m ? order : -order;
  const int along = by_m ? tiles_n : tiles_m;     // tiles walked per group member
  const int total = by_m ? tiles_m : tiles_n;     // tiles of the grouped dimension
  const int group = b / (g * along);
  const int first = group * g;
  const int gsz = min(total - first, g);
  const int in_g = b - group * g * along;
  const int grouped = first + in_g % gsz, walked = in_g / gsz;
  return by_m ? int2{grouped, walked} : int2{walked, grouped};   // (tm, tn)
}

// raw buffer descriptor over [base, base + 4 GiB): the launcher guarantees every offset fits 32 bits
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
}

// Grouped (mixture-of-experts) form of v10 (GRP): G row groups (experts) share one launch.  Group e
// owns rows [g_offs[e], g_offs[e+1]) of C, its M tiles are virtual tiles [g_tiles[e], g_tiles[e+1])
// (ceil of its rows / BM), its weight is W + e * g_wstride, and its A rows are either contiguous from
// row g_offs[e] of A or gathered: A row g_rows[g_offs[e] + i] (the token a routed entry came from, so
// the activations are never permuted in memory; one index load per staged row, at block start).  M is
// a bound on the rows (the launch covers ceil(M / BM) M tiles); blocks past g_tiles[G] exit before
// touching LDS.
template <int EPI, bool GRP = false>
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
  int ks = 0;
  if constexpr (EPI == EPI_F32) {                    // split-K: consecutive ids = the K slices of a tile
    ks = bid % ep.ksplit;
    bid /= ep.ksplit;
  }
  const int tiles_m = (M + BM - 1) / BM;
  const int tiles_n = N / BN;
  const int2 tmn = tile_of(bid, tiles_m, tiles_n, ep.order);
  int tm = tmn.x;
  const int tn = tmn.y;
  const half_t* Ag = A;
  const half_t* Wg = W;
  half_t* Cg = C;
  const int* rows = nullptr;
  if constexpr (GRP) {
    if (tm >= ep.g_tiles[ep.g_n]) return;          // past the last group's tiles: whole block exits
    int e = 0;
    while (ep.g_tiles[e + 1] <= tm) ++e;             // wave-uniform scan (empty groups own no tiles)
    const int r0 = ep.g_offs[e];
    M = ep.g_offs[e + 1] - r0;
    tm -= ep.g_tiles[e];
    Wg = W + (size_t)e * ep.g_wstride;
    Cg = C + (size_t)r0 * ldc;
    if (ep.g_rows) rows = ep.g_rows + r0;
    else Ag = A + (size_t)r0 * lda;
  }
  if constexpr (EPI == EPI_F32) {                    // this block's K slice; its own partial slab
    Ag += (size_t)ks * ep.kslice;
    Wg += (size_t)ks * ep.kslice;
    Cg = (half_t*)((float*)C + (size_t)ks * ep.part_stride);
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
  unsigned xo[8], wo[8];
  const size_t wb_off = (size_t)64 * ldw * 2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (GRP) {
      int ra = min(m0 + prow[i] + lr, M - 1), rb = min(m0 + prow[i] + 64 + lr, M - 1);
      if (rows) {
        ra = rows[ra];
        rb = rows[rb];
      }
      xo[i] = (unsigned)(ra * lda + lc * 8) * 2u;
      xo[4 + i] = (unsigned)(rb * lda + lc * 8) * 2u;
    } else {
      xo[i] = (unsigned)(min(m0 + prow[i] + lr, M - 1) * lda + lc * 8) * 2u;
      xo[4 + i] = (unsigned)(min(m0 + prow[i] + 64 + lr, M - 1) * lda + lc * 8) * 2u;
    }
    if constexpr (EPI == FLS_EPI_SWIGLU) {
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        const int l = prow[i] + hb * 64;
        wo[hb * 4 + i] = (unsigned)((((l >> 4) & 1) * ep.gu_rows + (l >> 5) * 16 + (l & 15) + lr) * ldw + lc * 8) * 2u;
      }
    } else {
      wo[i] = (unsigned)((prow[i] + lr) * ldw + lc * 8) * 2u;
    }
  }
  const char* Ab = (const char*)Ag;
  const char* Wb = (const char*)(Wg + (size_t)(EPI == FLS_EPI_SWIGLU ? n0 / 2 : n0) * ldw);
  const __amdgpu_buffer_rsrc_t rA = make_rsrc(Ab);
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(Wb);
  const __amdgpu_buffer_rsrc_t rZ = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(Ab), (short)0, 0, 0x00020000);
// LDS-DMA of one 1 KiB piece: buffer_load ... lds with the per-lane 32-bit offset and the K (and
// half-tile) step in soffset (0.5-1% over the global_load_lds form, profiles/r2_gemm)
#define V10_DMA_X(rs, k0, idx, dst)                                                                \
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)(dst), 16, xo[idx], (k0) * 2, 0, 0)
#define V10_DMA_W(rs, hb, i, k0, dst)                                                              \
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)(dst), 16,                             \
      EPI == FLS_EPI_SWIGLU ? wo[(hb) * 4 + (i)] : wo[(i)],                                         \
      (EPI == FLS_EPI_SWIGLU ? 0u : (unsigned)((hb) * wb_off)) + (k0) * 2, 0, 0)
#define V10_X(buf, hb, k0)                                                                         \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                \
    V10_DMA_X(rA, k0, (hb) * 4 + i_, smem + (buf) * BUF + (prow[i_] + (hb) * 64) * 128);
#define V10_W(buf, hb, k0)                                                                         \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                \
    V10_DMA_W(rW, hb, i_, k0, smem + (buf) * BUF + WIMG + (prow[i_] + (hb) * 64) * 128);

  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, grp = lane >> 4;
  const int sw = fr & 7;
  const int c0 = ((0 + grp) ^ sw) << 4;
  const int c1 = ((4 + grp) ^ sw) << 4;
  const int xrow = (wm * 128 + fr) * 128;
  const int wrow = WIMG + (wn * 128 + fr) * 128;

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
    xf[u_][0] = *(const half8*)(smem + (buf) * BUF + xrow + u_ * 2048 + c0);                      \
    xf[u_][1] = *(const half8*)(smem + (buf) * BUF + xrow + u_ * 2048 + c1);                      \
  }
#define V10_RW(buf, h)                                                                             \
  _Pragma("unroll") for (int t_ = (h) * 4; t_ < (h) * 4 + 4; ++t_) {                              \
    wf[t_][0] = *(const half8*)(smem + (buf) * BUF + wrow + t_ * 2048 + c0);                      \
    wf[t_][1] = *(const half8*)(smem + (buf) * BUF + wrow + t_ * 2048 + c1);                      \
  }
// one phase: 32 MFMAs (k-step outer, 4x4 tiles of the quadrant) with, in issue order,
// one ds_read after each of the first 16 even-numbered MFMAs and the half-tile's 4
// LDS-DMA ops after MFMAs 17, 20, 23, 26; then lgkmcnt(0) + counted vmcnt + barrier.
// RX: 1 = read an X half, 0 = a W half.
#define V10_PHASE(xh, wh, RX, rbuf, rh, DX, dbuf, dhb, dk0, SYNC)                                  \
  {                                                                                               \
    _Pragma("unroll") for (int i_ = 0; i_ < 32; ++i_) {                                           \
      const int s_ = i_ >> 4, u_ = (xh) * 4 + ((i_ >> 2) & 3), t_ = (wh) * 4 + (i_ & 3);          \
      mfma_acc_inplace_ordered(acc[u_][t_], wf[t_][s_], xf[u_][s_]);                              \
      if (i_ < 16 && (i_ & 1) == 0) {                                                             \
        const int rj_ = i_ >> 1;                                                                  \
        const int f_ = (rh) * 4 + (rj_ >> 1), k_ = rj_ & 1;                                       \
        if (RX)                                                                                   \
          xf[f_][k_] = *(const half8*)(smem + (rbuf) * BUF + xrow + f_ * 2048 + (k_ ? c1 : c0));  \
        else                                                                                      \
          wf[f_][k_] = *(const half8*)(smem + (rbuf) * BUF + wrow + f_ * 2048 + (k_ ? c1 : c0));  \
      }                                                                                           \
      if (i_ >= 17 && i_ <= 26 && (i_ - 17) % 3 == 0) {                                           \
        const int p_ = (i_ - 17) / 3;                                                             \
        if (DX)                                                                                   \
          V10_DMA_X(rX##dk0, dk0, (dhb) * 4 + p_, smem + (dbuf) * BUF + (prow[p_] + (dhb) * 64) * 128); \
        else                                                                                      \
          V10_DMA_W(rW##dk0, dhb, p_, dk0, smem + (dbuf) * BUF + WIMG + (prow[p_] + (dhb) * 64) * 128); \
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
    // past the last K-tile the DMA goes through a 0-record descriptor: issued and counted by
    // vmcnt like the others, but it moves no bytes (1.6% of the L2 reads at K = 8192)
    const __amdgpu_buffer_rsrc_t rXka = kt + 2 < nk ? rA : rZ, rWka = kt + 2 < nk ? rW : rZ;
    const __amdgpu_buffer_rsrc_t rXkb = kt + 3 < nk ? rA : rZ, rWkb = kt + 3 < nk ? rW : rZ;
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
#undef V10_RW
#undef V10_RX
#undef V10_W
#undef V10_X
#undef V10_DMA_X
#undef V10_DMA_W

  epilogue_quadrant<EPI>(Cg, ldc, M, m0 + wm * 128 + fr, n0 + wn * 128, grp, acc, ep);
}

#undef V10_PHASE

// Default tile order (profiles/r2_gemm/README.md).  Groups of g tiles of one dimension are walked
// along the other; the XCD remap gives XCD x the virtual ids [x*q, (x+1)*q), q = tiles / 8.
//  * 4 <= g <= 8 keeps an XCD's 32 concurrent tiles a compact g x 32/g block (11-12 operand panels
//    per K-step in its L2);
//  * g dividing tiles/8 along the grouped dimension gives every XCD whole groups, so all XCDs walk
//    the other operand in step and the MALL serves each of its panels to all 8 (N-grouped: the
//    activations; each XCD keeps its own chunk of the weight).
// Measured on the 70B shapes at 14k rows: N-grouped -4 (O, down, gate/up) and -5 (QKV) beat
// round 1's fixed orders by 0.5-2.5% and the M-grouped lock-step order 7 by 1-2%.
int auto_order(int tiles_m, int tiles_n) {
  if (tiles_n % 8 == 0)
    for (int g = 4; g <= 8; ++g)
      if ((tiles_n / 8) % g == 0) return -g;
  if (tiles_m % 8 == 0)
    for (int g = 4; g <= 8; ++g)
      if ((tiles_m / 8) % g == 0) return g;
  return -4;
}

}  // namespace
