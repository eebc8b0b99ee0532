// Shared-prefix / varlen flash attention forward on gfx950 (MI355X).
//
// Replaces the reference's eager attention (HF LlamaAttention via
// utils.py:272-279): prefix K/V expanded to every suffix, concatenated, then
// repeat_kv'd to every query head — materialised n_s * (nh/nkv) times — and a
// [1, nh, Lp, Lp] fp32 probability matrix.
//
// Here K/V are read IN PLACE from the packed QKV activation.  A work item
// (runtime/batch.py) is a block of <= q_block query rows plus up to two key ranges
//   range 0: the prompt's shared prefix (bidirectional, or causal for prefix
//            queries in --prefix_attention causal),
//   range 1: suffix rows, causal and block-diagonal: key j is visible to query
//            row i iff seg_lo[i] <= j <= i (packed rows; seg_lo = first row of
//            the suffix holding row i),
// so one item can hold several suffixes of one prompt and they all read the
// prompt's single prefix K/V in the same pass (GQA-native: query head h uses
// kv head h / (nh/nkv)).  Without seg_lo an item's range 1 is one suffix.
//
// Block: HPB query heads of one KV group x WPH waves of 32 query rows each
// (q_block = 32 * WPH); every K/V tile staged in LDS feeds HPB * WPH waves.
//   * S^T = K . Q^T with v_mfma_f32_16x16x32_f16 (A = K fragment from LDS,
//     B = Q fragment in registers): each lane owns one query row's 16 scores
//     of a 64-key tile, so the row max is in-lane + two permlane swaps and the
//     P fragment of the next MFMA is lane-local;
//   * O^T += V^T . P^T with V^T from ds_read_b64_tr_b16 (hardware transpose
//     read) of a row-major, XOR-swizzled V tile; K tile XOR-swizzled per
//     16-byte chunk for conflict-free ds_read_b128;
//   * K/V tiles register-staged (32-bit buffer loads issued one tile ahead,
//     written to the other LDS buffer after the tile's MFMAs): one barrier per
//     tile (guide T14);
//   * softmax VALU work kept off the MFMA critical path: raw scores (the scale
//     folds into one FMA per score before the exp), masking only on boundary
//     tiles (wave-uniform branch), max3 chains without canonicalisation, and a
//     deferred rescale (guide T13): O and l are rescaled only when a row's max
//     grows by more than 2^8, otherwise P is taken against the old max
//     (P <= 256: exact range in fp16; O and l accumulate in fp32).
// Measured (profiles/r2_attn): 70B heads, 1k prefix + 5 x 64 suffixes 828
// TFLOP/s (round-1 kernel 728), 4k prefix 992 (880).
#include "common.h"
#include "fls.h"

namespace {

constexpr int KT = 64;                 // keys per tile
constexpr float DEFER_LOG2 = 8.0f;     // deferred-rescale threshold (log2 units)

template <int HD>
struct Lds {
  static constexpr int ROW = HD * 2;            // bytes per row
  static constexpr int NCH = HD / 8;            // 16-byte chunks per row
  // XOR masks stay inside the row: all chunk bits for power-of-two rows (hd 64 / 128), the low two
  // bits for hd 96 (12 chunks: an XOR within each aligned group of 4 chunks)
  static constexpr int KM = (NCH & (NCH - 1)) == 0 ? NCH - 1 : 3;
  static constexpr int VM = (NCH & (NCH - 1)) == 0 ? NCH / 2 - 1 : 1;
  // K: ds_read_b128 row reads -> chunk ^ (row & KM)
  __device__ static int k_off(int row, int ch) { return row * ROW + ((ch ^ (row & KM)) << 4); }
  // V: ds_read_b64_tr_b16 -> chunk ^ ((row & VM) << 1)
  __device__ static int v_off(int row, int ch) { return row * ROW + ((ch ^ ((row & VM) << 1)) << 4); }
};

// max without the canonicalising v_max(x, x) the compiler puts in front of fmaxf on MFMA results
// (guide: keep such ops single instructions); scores are never NaN here
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// max over the 4 lane groups (lanes l, l^16, l^32, l^48) that hold one query row: VALU permlane
// swaps, not ds_bpermute (the LDS pipe is busy with the K / V^T fragment reads)
__device__ __forceinline__ float max_xor16_32(float v) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = vmax(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return vmax(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

typedef float float2_ __attribute__((ext_vector_type(2)));
template <int N>
struct IC {
  static constexpr int value = N;
};
typedef _Float16 half2_ __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned pack_h2(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(float2_{a, b}, half2_));
}

// ds_read_b64_tr_b16 without the compiler's wait: its builtin makes the compiler drain every
// outstanding LDS-DMA (vmcnt(0)) in front of the read.  The caller waits with lds_wait4 before
// using the result (the wait's in/out operands order every use after it).
__device__ __forceinline__ half4 lds_tr16_async(const char* p) {
  half4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"((unsigned)(uintptr_t)(const LDS_AS char*)p) : "memory");
  return v;
}
__device__ __forceinline__ void lds_wait4(half4& a, half4& b, half4& c, half4& d, half4& e, half4& f, half4& g,
                                          half4& h) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)::"memory");
}

// SPL (split-KV, R2 only): blockIdx.z walks one of gridDim.z contiguous slices of the item's key
// tiles and writes its unnormalised O, running max and row sum in fp32 to `part`
// ([rows][splits][nh] x (HD + 2)); attn_split_combine merges the slices.  For grids with fewer
// blocks than CUs (few prompts with long contexts), which otherwise leave most CUs idle.
template <int HD, int HPB, int WPH, bool R2, bool SPL = false>
__global__ __launch_bounds__(64 * WPH * HPB, 2) void attn_fwd(const half_t* __restrict__ qkv, half_t* __restrict__ out,
                                                    const int* __restrict__ work, const int* __restrict__ seg_lo,
                                                    int nh, int nkv, int ld_qkv, int ld_out, float scale_log2,
                                                    const half_t* __restrict__ kv0, int ld_kv0,
                                                    const int* __restrict__ work2, const int* __restrict__ r2win,
                                                    float* __restrict__ part) {
  static_assert(!SPL || R2, "split-KV is built for the range-2 (suffix K/V reuse) kernel only");
  constexpr int NT_ = 64 * WPH * HPB;
  constexpr int NS = HD / 32;               // k-steps of QK^T
  constexpr int NU = HD / 16;               // 16-wide d subtiles of O
  constexpr int CH = HD / 8;                // 16-byte chunks per K/V row
  constexpr int PER = KT * CH / NT_;        // chunks per thread per operand
  static_assert(PER >= 1 && (KT * CH) % NT_ == 0, "tile / block mismatch");
  constexpr int TILE_BYTES = 2 * KT * HD * 2;         // K + V
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: h, g, descriptors in SGPRs
  const int h = blockIdx.y * HPB + wave / WPH;
  const int g = h / (nh / nkv);             // same for every head of the block (HPB | group)
  const int rbase = (wave % WPH) * 32;      // this wave's first query row of the item

  const int* wi = work + blockIdx.x * 8;
  const int q_start = wi[0], q_len = wi[1], q_off = wi[2];
  if (q_len <= 0) return;                   // padding item (bucketed graph replays); block-uniform
  const int r_start0 = wi[3], r_len0 = wi[4], r_causal0 = wi[5];
  const int r_start1 = wi[6], r_len1 = wi[7];
  const int kend0 = r_len0 <= 0 ? 0 : (r_causal0 ? min(r_len0, q_off + q_len) : r_len0);
  // R2 (suffix K/V reuse): every key of a suffix, the new rows' included, is read from the cache
  // as range 2 through per-row windows, so there is no range 1
  const int kend1 = (R2 || r_len1 <= 0) ? 0 : min(r_len1, q_off + q_len);
  const int n0 = (kend0 + KT - 1) / KT;
  // R2: range 2 = rows [r_start2, r_start2 + r_len2) of kv0 (a suffix's cached K/V), all visible,
  // walked between range 0 and range 1
  int r_start2 = 0, r_len2 = 0;
  if constexpr (R2) {
    r_start2 = work2[blockIdx.x * 2];
    r_len2 = max(work2[blockIdx.x * 2 + 1], 0);
  }
  const int n02 = n0 + (r_len2 + KT - 1) / KT;
  const int ntiles = n02 + (kend1 + KT - 1) / KT;
  // this block's key tiles [t_lo, t_hi): all of them unless split
  int t_lo = 0, t_hi = ntiles;
  if constexpr (SPL) {
    const int per = (ntiles + (int)gridDim.z - 1) / (int)gridDim.z;
    t_lo = min(ntiles, (int)blockIdx.z * per);
    t_hi = min(ntiles, t_lo + per);
  }

  const int fr = lane & 15, grp = lane >> 4;
  const int k_col = nh * HD + g * HD;
  const int v_col = (nh + nkv) * HD + g * HD;
  // one buffer descriptor per key range, based at the range's first row: 32-bit offsets
  // (klen * ld * 2 bytes stays far below 4 GiB for any context this engine accepts)
  const bool cache0 = kv0 != nullptr;                  // range 0 from the prefix K/V cache
  const int ld0 = cache0 ? ld_kv0 : ld_qkv;
  const int kc0 = cache0 ? g * HD : k_col, vc0 = cache0 ? (nkv + g) * HD : v_col;
  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<half_t*>((cache0 ? kv0 : qkv) + (size_t)r_start0 * ld0), (short)0, -1, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<half_t*>(qkv + (size_t)r_start1 * ld_qkv), (short)0, -1, 0x00020000);
  // range 2 rows lie after range 0's in the same cache buffer: read through rs0 at a row offset (a
  // third descriptor in the tile loader's select costs registers the R2 kernel does not have)
  const int r2base = R2 ? r_start2 - r_start0 : 0;

  half8 qf[2][NS];
  int qi[2], lo[2], lo2[2] = {0, 0}, hi2[2] = {0, 0};
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int qrow = rbase + qg * 16 + fr;
    const int qr = q_start + min(qrow, q_len - 1);
    const half_t* qp = qkv + (size_t)qr * ld_qkv + h * HD + grp * 8;
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[qg][s] = *(const half8*)(qp + s * 32);
    qi[qg] = q_off + qrow;                  // range-1 index of this query row (causal upper bound)
    lo[qg] = seg_lo && r_len1 > 0 ? seg_lo[qr] - r_start1 : 0;   // its suffix's first range-1 key
    if constexpr (R2) {                     // its suffix's window of range 2 (relative rows)
      lo2[qg] = r2win[2 * qr] - r_start2;
      hi2[qg] = r2win[2 * qr + 1] - r_start2;
    }
  }
  // the wave's first query row bounds every causal compare from below: a tile is fully visible to
  // the whole wave iff its last key is visible to that row (range 1 with several suffixes: masked)
  const int qi_min = q_off + rbase;
  const bool multi = seg_lo != nullptr;
  const int live_rows = q_len - rbase;      // query rows of this wave inside the item (uniform)

  floatx4 o[2][NU];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg)
#pragma unroll
    for (int u = 0; u < NU; ++u) o[qg][u] = floatx4{0.f, 0.f, 0.f, 0.f};
  float m_run[2] = {-1e30f, -1e30f};        // raw-score domain
  float l_run[2] = {0.f, 0.f};

  u32x4 pk[PER], pv[PER];
  // tile loader: by-reference captures for the plain kernel (its tuned code), by-value for R2 (whose
  // three-range selects otherwise keep the captured locals in scratch memory)
#define FLS_ATTN_LOAD_TILE_BODY \
    const bool r1 = t >= n02; \
    const bool r2 = R2 && !r1 && t >= n0; \
    const int k0 = (r1 ? t - n02 : (r2 ? t - n0 : t)) * KT; \
    const int klen = r1 ? r_len1 : (r2 ? r_len2 : r_len0); \
    const int ldk = r1 ? ld_qkv : ld0; \
    const int rb = r2 ? r2base : 0; \
    const unsigned kc = (unsigned)(r1 ? k_col : kc0) * 2u, vc = (unsigned)(r1 ? v_col : vc0) * 2u; \
    const __amdgpu_buffer_rsrc_t r = r1 ? rs1 : rs0; \
_Pragma("unroll") \
    for (int i = 0; i < PER; ++i) { \
      const int c = tid + i * NT_; \
      const int row = c / CH, ch = c % CH; \
      const unsigned off = (unsigned)((rb + min(k0 + row, klen - 1)) * ldk + ch * 8) * 2u; \
      K_[i] = __builtin_amdgcn_raw_buffer_load_b128(r, off, kc, 0); \
      V_[i] = __builtin_amdgcn_raw_buffer_load_b128(r, off, vc, 0); \
    }
  auto load_tile_ref = [&](int t) { u32x4(&K_)[PER] = pk; u32x4(&V_)[PER] = pv; FLS_ATTN_LOAD_TILE_BODY };
  auto load_tile_val = [=, &pk, &pv](int t) { u32x4(&K_)[PER] = pk; u32x4(&V_)[PER] = pv; FLS_ATTN_LOAD_TILE_BODY };
#undef FLS_ATTN_LOAD_TILE_BODY
  auto load_tile = [&](int t) {
    if constexpr (R2) load_tile_val(t);
    else load_tile_ref(t);
  };
  auto store_tile = [&](int buf) {
    char* Ks = smem + buf * TILE_BYTES;
    char* Vs = Ks + KT * HD * 2;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NT_;
      const int row = c / CH, ch = c % CH;
      *(u32x4*)(Ks + Lds<HD>::k_off(row, ch)) = pk[i];
      *(u32x4*)(Vs + Lds<HD>::v_off(row, ch)) = pv[i];
    }
  };

  // per-tile key range of tile t
#define FLS_ATTN_TILE_PRE \
    const bool r1 = t >= n02; \
    const bool r2 = R2 && !r1 && t >= n0; \
    const int k0 = (r1 ? t - n02 : (r2 ? t - n0 : t)) * KT; \
    const int klen = r1 ? r_len1 : (r2 ? r_len2 : r_len0); \
    const bool causal = r1 || (!r2 && r_causal0); \
    const char* Ks = smem + (t & 1) * TILE_BYTES; \
    const char* Vs = Ks + KT * HD * 2;

    // the tile's math for the wave's first NQ 16-row query groups (NQ = 2: the whole wave)
#define FLS_ATTN_TILE_MATH \
    /* ---- S^T = K Q^T for both 16-row query groups (each K fragment read once) */ \
    floatx4 sc[2][4]; \
_Pragma("unroll") \
    for (int tt = 0; tt < 4; ++tt) { \
      sc[0][tt] = floatx4{0.f, 0.f, 0.f, 0.f}; \
      if constexpr (NQ > 1) sc[1][tt] = floatx4{0.f, 0.f, 0.f, 0.f}; \
      const int krow = tt * 16 + fr; \
_Pragma("unroll") \
      for (int s = 0; s < NS; ++s) { \
        const half8 kf = *(const half8*)(Ks + Lds<HD>::k_off(krow, s * 4 + grp)); \
        sc[0][tt] = mfma16x16x32(kf, qf[0][s], sc[0][tt]); \
        if constexpr (NQ > 1) sc[1][tt] = mfma16x16x32(kf, qf[1][s], sc[1][tt]); \
      } \
    } \
    FLS_ATTN_AFTER_QK \
    /* ---- visibility: wave-uniform fast path when every key of the tile is visible to every row */ \
    const int vis_last = causal ? min(klen - 1, qi_min) : klen - 1; \
    if (k0 + KT - 1 > vis_last || (r1 && multi) || r2) { \
      asm volatile("" ::: "memory");        /* keep this a branch (not per-score selects on every tile) */ \
_Pragma("unroll") \
      for (int qg = 0; qg < NQ; ++qg) { \
        /* key k0 + 16tt + 4grp + r is visible iff lo_rel <= 16tt + r <= hi_rel */ \
        const int hi_rel = (r2 ? min(klen, hi2[qg]) - 1 : (causal ? min(klen - 1, qi[qg]) : klen - 1)) - k0 - grp * 4; \
        const int lo_rel = (r1 ? lo[qg] : (r2 ? lo2[qg] : 0)) - k0 - grp * 4; \
_Pragma("unroll") \
        for (int tt = 0; tt < 4; ++tt) \
_Pragma("unroll") \
          for (int r = 0; r < 4; ++r) \
            if (tt * 16 + r > hi_rel || tt * 16 + r < lo_rel) sc[qg][tt][r] = -INFINITY; \
      } \
    } \
    /* ---- online softmax per query group */ \
    half8 pf[2][2]; \
_Pragma("unroll") \
    for (int qg = 0; qg < NQ; ++qg) { \
      /* 16 scores of this lane's query: two independent max3 chains, then across the lane groups */ \
      float ma = vmax3(sc[qg][0][0], sc[qg][0][1], sc[qg][0][2]); \
      float mb = vmax3(sc[qg][2][0], sc[qg][2][1], sc[qg][2][2]); \
      ma = vmax3(ma, sc[qg][0][3], sc[qg][1][0]); \
      mb = vmax3(mb, sc[qg][2][3], sc[qg][3][0]); \
      ma = vmax3(ma, sc[qg][1][1], sc[qg][1][2]); \
      mb = vmax3(mb, sc[qg][3][1], sc[qg][3][2]); \
      const float mx = max_xor16_32(vmax3(ma, sc[qg][1][3], vmax(mb, sc[qg][3][3]))); \
      /* deferred rescale: keep the old max unless some row of the wave grew past 2^DEFER_LOG2 */ \
      /* (the previous tile's P.V is complete: nothing at the old scale is pending) */ \
      /* (each row decides for itself: a row's result never depends on the other rows of its wave, */ \
      /* so a generation step reusing cached K/V is bitwise the full re-computation: alpha = 1 exactly */ \
      /* for the rows that keep their max) */ \
      if (!__all((mx - m_run[qg]) * scale_log2 <= DEFER_LOG2)) { \
        const float m_new = (mx - m_run[qg]) * scale_log2 > DEFER_LOG2 ? mx : m_run[qg]; \
        const float alpha = fast_exp2((m_run[qg] - m_new) * scale_log2); \
        l_run[qg] *= alpha; \
_Pragma("unroll") \
        for (int u = 0; u < NU; ++u) o[qg][u] *= alpha; \
        m_run[qg] = m_new; \
      } \
      const float mc = m_run[qg] * scale_log2; \
      float psum = 0.f; \
      unsigned pw[8]; \
_Pragma("unroll") \
      for (int tt = 0; tt < 4; ++tt) { \
        float p[4]; \
_Pragma("unroll") \
        for (int r = 0; r < 4; ++r) { \
          p[r] = fast_exp2(__builtin_fmaf(sc[qg][tt][r], scale_log2, -mc)); \
          psum += p[r]; \
        } \
        pw[tt * 2] = pack_h2(p[0], p[1]); \
        pw[tt * 2 + 1] = pack_h2(p[2], p[3]); \
      } \
      l_run[qg] += psum; \
      /* P^T fragment: element (tt & 1) * 4 + r of k-step tt >> 1 = key 16 tt + 4 grp + r */ \
_Pragma("unroll") \
      for (int ks = 0; ks < 2; ++ks) \
        pf[qg][ks] = __builtin_bit_cast(half8, u32x4{pw[ks * 4], pw[ks * 4 + 1], pw[ks * 4 + 2], pw[ks * 4 + 3]}); \
    } \
    /* ---- O^T += V^T P^T (each V^T fragment read once for both groups) */ \
    const int q4 = (lane & 15) >> 2, p4 = lane & 3; \
_Pragma("unroll") \
    for (int ks = 0; ks < 2; ++ks) { \
      const int row_a = ks * 32 + grp * 4 + q4; \
      const int row_b = row_a + 16; \
_Pragma("unroll") \
      for (int u = 0; u < NU; ++u) { \
        const int ch = u * 2 + (p4 >> 1); \
        const half4 va = ds_read_tr16(Vs + Lds<HD>::v_off(row_a, ch) + (p4 & 1) * 8); \
        const half4 vb = ds_read_tr16(Vs + Lds<HD>::v_off(row_b, ch) + (p4 & 1) * 8); \
        const half8 vf = {va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]}; \
        o[0][u] = mfma16x16x32(vf, pf[0][ks], o[0][u]); \
        if constexpr (NQ > 1) o[1][u] = mfma16x16x32(vf, pf[1][ks], o[1][u]); \
      } \
    }
#define FLS_ATTN_AFTER_QK
  if (t_hi > t_lo) {
    load_tile(t_lo);
    store_tile(t_lo & 1);
    if (t_hi > t_lo + 1) load_tile(t_lo + 1);
  }
  __syncthreads();
  for (int t = t_lo; t < t_hi; ++t) {
    FLS_ATTN_TILE_PRE
    if constexpr (!R2) {
      constexpr int NQ = 2;
      FLS_ATTN_TILE_MATH
    } else {
      // a decode-like item holds a few new rows (one per suffix): the waves and 16-row groups past
      // q_len skip their MFMAs and softmax (wave-uniform), instead of padding every item to q_block
      auto tile_math = [&](auto nq_c) {
        constexpr int NQ = decltype(nq_c)::value;
        FLS_ATTN_TILE_MATH
      };
      if (live_rows > 16) tile_math(IC<2>{});
      else if (live_rows > 0) tile_math(IC<1>{});
    }
    if (t + 1 < t_hi) {
      store_tile((t + 1) & 1);               // the other buffer's readers (tile t-1) passed the last barrier
      if (t + 2 < t_hi) load_tile(t + 2);    // in flight under tile t+1's MFMAs
    }
    __syncthreads();
  }
#undef FLS_ATTN_AFTER_QK
#undef FLS_ATTN_TILE_PRE
  // ---- normalise and store (split: the slice's fp32 partials)
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    float l = l_run[qg];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const int qrow = rbase + qg * 16 + fr;
    if constexpr (SPL) {
      if (qrow < q_len) {
        float* pp = part + ((size_t)((q_start + qrow) * (int)gridDim.z + (int)blockIdx.z) * nh + h) * (HD + 2);
#pragma unroll
        for (int u = 0; u < NU; ++u) *(floatx4*)(pp + u * 16 + grp * 4) = o[qg][u];
        if (grp == 0) *(float2_*)(pp + HD) = float2_{m_run[qg] * scale_log2, l};
      }
      continue;
    }
    if (qrow < q_len) {
      const float inv = 1.f / l;
      half_t* op = out + (size_t)(q_start + qrow) * ld_out + h * HD + grp * 4;
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        half4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (half_t)(o[qg][u][r] * inv);
        *(half4*)(op + u * 16) = v;
      }
    }
  }
}

// Persistent form of attn_fwd for the full-pass (no range 2, no split) items: a grid of about one
// block per CU slot walks work units u = blockIdx.x, + gridDim.x, ... where a unit is (work item,
// group of HPB query heads).  The K/V tile pipeline runs across unit boundaries: the register-staged
// loads of the next unit's first tiles are in flight under the current unit's last tiles, and the
// next unit's Q fragments are loaded right after the last tile's S = K Q^T MFMAs (Q is dead then),
// under that tile's softmax, P.V and the unit's output stores.  A 1k-token prefix item is only 16
// key tiles, so a block per unit exposed its start (Q load, first two tiles) and drain at every
// item (attn_fwd: 828 TFLOP/s at a 1k prefix vs 992 at 4k, profiles/r2_attn).
// Units in order u = item * (nh / HPB) + head group: with a grid that is a multiple of nh / HPB
// a block keeps one head group, and the blocks of one XCD (b mod 8) share a few KV heads' K/V in
// their L2.  Bitwise equal to attn_fwd (same per-tile arithmetic in the same order).
template <int HD, int HPB, int WPH>
__global__ __launch_bounds__(64 * WPH * HPB, 2) void attn_fwd_pers(const half_t* __restrict__ qkv,
                                                         half_t* __restrict__ out, const int* __restrict__ work,
                                                         const int* __restrict__ seg_lo, int nh, int nkv,
                                                         int ld_qkv, int ld_out, float scale_log2,
                                                         const half_t* __restrict__ kv0, int ld_kv0, int n_items) {
  constexpr bool R2 = false;
  constexpr int NT_ = 64 * WPH * HPB;
  constexpr int NS = HD / 32;
  constexpr int NU = HD / 16;
  constexpr int CH = HD / 8;
  constexpr int PER = KT * CH / NT_;
  static_assert(PER >= 1 && (KT * CH) % NT_ == 0, "tile / block mismatch");
  constexpr int TILE_BYTES = 2 * KT * HD * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hw = wave / WPH;                 // head of the block's group
  const int rbase = (wave % WPH) * 32;       // this wave's first query row of an item
  const int fr = lane & 15, grp = lane >> 4;
  const int n_hg = nh / HPB;
  const int n_units = n_items * n_hg;
  const int G = gridDim.x;
  const int hpg = nh / nkv;
  const bool cache0 = kv0 != nullptr;
  const int ld0 = cache0 ? ld_kv0 : ld_qkv;
  const bool multi = seg_lo != nullptr;

  // a unit's parameters (block-uniform: scalar loads of its work item)
  struct UP {
    int q_start, q_len, q_off, r_start0, r_len0, r_causal0, r_start1, r_len1, hg, n0, ntiles;
  };
  auto unit = [&](int u) {
    UP p;
    const int* wi = work + (u / n_hg) * 8;
    p.hg = u % n_hg;
    p.q_start = wi[0];
    p.q_len = wi[1];
    p.q_off = wi[2];
    p.r_start0 = wi[3];
    p.r_len0 = wi[4];
    p.r_causal0 = wi[5];
    p.r_start1 = wi[6];
    p.r_len1 = wi[7];
    const int kend0 = p.r_len0 <= 0 ? 0 : (p.r_causal0 ? min(p.r_len0, p.q_off + p.q_len) : p.r_len0);
    const int kend1 = p.r_len1 <= 0 ? 0 : min(p.r_len1, p.q_off + p.q_len);
    p.n0 = (kend0 + KT - 1) / KT;
    p.ntiles = p.q_len <= 0 ? 0 : p.n0 + (kend1 + KT - 1) / KT;
    return p;
  };
  auto next_valid = [&](int u) {
    while (u < n_units && unit(u).ntiles <= 0) u += G;   // padding items (q_len 0) have no tiles
    return u;
  };

  int mu = next_valid((int)blockIdx.x);
  if (mu >= n_units) return;                 // block-uniform
  UP M = unit(mu);

  half8 qf[2][NS];
  int qi[2], lo[2];
  const int lo2[2] = {0, 0}, hi2[2] = {0, 0};
  auto load_q = [&](const UP& p) {
    const int h = p.hg * HPB + hw;
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
      const int qr = p.q_start + min(rbase + qg * 16 + fr, p.q_len - 1);
      const half_t* qp = qkv + (size_t)qr * ld_qkv + h * HD + grp * 8;
#pragma unroll
      for (int s = 0; s < NS; ++s) qf[qg][s] = *(const half8*)(qp + s * 32);
    }
  };
  auto unit_rows = [&](const UP& p) {
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
      const int qrow = rbase + qg * 16 + fr;
      const int qr = p.q_start + min(qrow, p.q_len - 1);
      qi[qg] = p.q_off + qrow;
      lo[qg] = multi && p.r_len1 > 0 ? seg_lo[qr] - p.r_start1 : 0;
    }
  };

  // the load cursor: unit lu (parameters L), tile lt
  int lu = mu, lt = 0;
  UP L = M;
  u32x4 pk[PER], pv[PER];
  auto load_tile = [&]() {
    const int g = (L.hg * HPB) / hpg;
    const int k_col = nh * HD + g * HD, v_col = (nh + nkv) * HD + g * HD;
    const bool r1 = lt >= L.n0;
    const int k0 = (r1 ? lt - L.n0 : lt) * KT;
    const int klen = r1 ? L.r_len1 : L.r_len0;
    const int ldk = r1 ? ld_qkv : ld0;
    const unsigned kc = (unsigned)(r1 ? k_col : (cache0 ? g * HD : k_col)) * 2u;
    const unsigned vc = (unsigned)(r1 ? v_col : (cache0 ? (nkv + g) * HD : v_col)) * 2u;
    const half_t* base = r1 ? qkv + (size_t)L.r_start1 * ld_qkv : (cache0 ? kv0 : qkv) + (size_t)L.r_start0 * ld0;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<half_t*>(base), (short)0, -1,
                                                                       0x00020000);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NT_;
      const int row = c / CH, ch = c % CH;
      const unsigned off = (unsigned)(min(k0 + row, klen - 1) * ldk + ch * 8) * 2u;
      pk[i] = __builtin_amdgcn_raw_buffer_load_b128(r, off, kc, 0);
      pv[i] = __builtin_amdgcn_raw_buffer_load_b128(r, off, vc, 0);
    }
    if (++lt >= L.ntiles) {                  // advance the cursor (uniform)
      lu = next_valid(lu + G);
      lt = 0;
      if (lu < n_units) L = unit(lu);
    }
  };
  auto store_tile = [&](int buf) {
    char* Ks = smem + buf * TILE_BYTES;
    char* Vs = Ks + KT * HD * 2;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NT_;
      const int row = c / CH, ch = c % CH;
      *(u32x4*)(Ks + Lds<HD>::k_off(row, ch)) = pk[i];
      *(u32x4*)(Vs + Lds<HD>::v_off(row, ch)) = pv[i];
    }
  };

  // static priority for the second-dispatched half of the 8 waves (MI355X_MICROARCH: the younger half
  // loses every VALU arbitration otherwise): +0.5% at the 70B headline shape (profiles/r6_attn)
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  load_q(M);
  unit_rows(M);
  load_tile();                               // step 0
  store_tile(0);
  bool have = lu < n_units;                  // the registers hold the next step's tile
  if (have) load_tile();                     // step 1
  __syncthreads();

  int s = 0;                                 // global step (LDS buffer parity)
  for (;;) {
    floatx4 o[2][NU];
#pragma unroll
    for (int qg = 0; qg < 2; ++qg)
#pragma unroll
      for (int u = 0; u < NU; ++u) o[qg][u] = floatx4{0.f, 0.f, 0.f, 0.f};
    float m_run[2] = {-1e30f, -1e30f};
    float l_run[2] = {0.f, 0.f};
    const int nu = next_valid(mu + G);       // the next unit of this block (uniform)
    const int qi_min = M.q_off + rbase;
    for (int mt = 0; mt < M.ntiles; ++mt, ++s) {
      const bool last = mt == M.ntiles - 1;
      const bool r1 = mt >= M.n0;
      const bool r2 = false;
      const int k0 = (r1 ? mt - M.n0 : mt) * KT;
      const int klen = r1 ? M.r_len1 : M.r_len0;
      const bool causal = r1 || M.r_causal0;
      const char* Ks = smem + (s & 1) * TILE_BYTES;
      const char* Vs = Ks + KT * HD * 2;
      constexpr int NQ = 2;
      // the next unit's Q, in flight under this tile's softmax and P.V and the output stores
#define FLS_ATTN_AFTER_QK \
      if (last && nu < n_units) load_q(unit(nu));
      FLS_ATTN_TILE_MATH
#undef FLS_ATTN_AFTER_QK
      if (have) {
        store_tile((s + 1) & 1);             // the other buffer's readers (step s-1) passed the barrier
        have = lu < n_units;
        if (have) load_tile();               // step s+2, in flight under step s+1's MFMAs
      }
      __syncthreads();
    }
    // ---- normalise and store this unit's rows
    const int h = M.hg * HPB + hw;
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
      float l = l_run[qg];
      l += __shfl_xor(l, 16, 64);
      l += __shfl_xor(l, 32, 64);
      const int qrow = rbase + qg * 16 + fr;
      if (qrow < M.q_len) {
        const float inv = 1.f / l;
        half_t* op = out + (size_t)(M.q_start + qrow) * ld_out + h * HD + grp * 4;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          half4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (half_t)(o[qg][u][r] * inv);
          *(half4*)(op + u * 16) = v;
        }
      }
    }
    if (nu >= n_units) break;
    mu = nu;
    M = unit(mu);
    unit_rows(M);
  }
}
#undef FLS_ATTN_TILE_MATH

// merge the split-KV slices of every row of every item: O = sum_z 2^(m_z - M) O_z / sum_z 2^(m_z - M) l_z
// (m in the log2 domain); block = one (item, head), a thread per head-dim column
template <int HD>
__global__ __launch_bounds__(HD) void attn_split_combine(const float* __restrict__ part, half_t* __restrict__ out,
                                                         const int* __restrict__ work, int nh, int ld_out, int ns) {
  const int* wi = work + blockIdx.x * 8;
  const int q_start = wi[0], q_len = wi[1];
  const int h = blockIdx.y, d = threadIdx.x;
  for (int r = 0; r < q_len; ++r) {
    const float* pp = part + ((size_t)(q_start + r) * ns * nh + h) * (HD + 2);
    const size_t zs = (size_t)nh * (HD + 2);
    float M = -INFINITY;
    for (int z = 0; z < ns; ++z) M = fmaxf(M, pp[z * zs + HD]);
    float L = 0.f, acc = 0.f;
    for (int z = 0; z < ns; ++z) {
      const float w = fast_exp2(pp[z * zs + HD] - M);
      L += w * pp[z * zs + HD + 1];
      acc += w * pp[z * zs + d];
    }
    out[(size_t)(q_start + r) * ld_out + h * HD + d] = (half_t)(acc / L);
  }
}

// Packed-GQA decode attention: range-2 items of a few query rows (generation steps with the prefix
// + suffix K/V caches, q_block 8).  One block = one (item, KV group).  The group's hpg query heads
// x q_len rows are packed into the N dimension of S^T = K.Q^T (packed row p = head hh * q_len +
// row r), 16 per wave, 64 per pass of the block's 4 waves: each K/V tile is read from HBM once per
// block and from LDS once per 16 packed rows, where the one-wave-per-head kernel reads it once
// per head and runs 5 live rows padded to 16 (profiles/r4_gen/attn_pmc).
//   * K/V tiles by LDS-DMA into an NB-deep ring, NB - 1 tiles in flight under the math of one;
//     the source chunk order pre-applies the XOR swizzle of the ds_read_b128 K and
//     ds_read_b64_tr_b16 V^T reads; one counted vmcnt + barrier per tile;
//   * the softmax and O^T += V^T.P^T steps are attn_fwd's (deferred rescale, lane-local P^T).
// SPL: blockIdx.z takes one of gridDim.z contiguous slices of the key tiles and writes fp32
// partials in attn_split_combine's layout.
template <int HD, bool SPL, int NB>
__global__ __launch_bounds__(256, 1) void attn_decode(const half_t* __restrict__ qkv, half_t* __restrict__ out,
                                                    const int* __restrict__ work, int nh, int nkv, int ld_qkv,
                                                    int ld_out, float scale_log2, const half_t* __restrict__ kv0,
                                                    int ld_kv0, const int* __restrict__ work2,
                                                    const int* __restrict__ r2win, float* __restrict__ part) {
  constexpr int NW = 4;                     // waves per block (16 packed rows each)
  // NB: tile ring depth (NB - 1 tiles in flight under the math of one)
  constexpr int NS = HD / 32;               // k-steps of QK^T
  constexpr int NU = HD / 16;               // 16-wide d subtiles of O
  constexpr int CH = HD / 8;                // 16-byte chunks per K/V row
  constexpr int TB = KT * HD * 2;           // one operand tile (16 KB at hd 128)
  constexpr int RPI = 64 / CH;              // rows per 1 KB DMA instruction
  constexpr int NI = TB / 1024 / NW;        // DMA instructions per wave per operand tile
  static_assert(NI >= 1 && NI * NW * 1024 == TB, "tile / block mismatch");
  __shared__ __attribute__((aligned(16))) char smem[NB * 2 * TB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = blockIdx.y;
  const int hpg = nh / nkv;
  const int* wi = work + blockIdx.x * 8;
  const int q_start = wi[0], q_len = wi[1], q_off = wi[2];
  if (q_len <= 0) return;                   // padding item; block-uniform
  const int r_start0 = wi[3], r_len0 = wi[4], r_causal0 = wi[5];
  const int kend0 = r_len0 <= 0 ? 0 : (r_causal0 ? min(r_len0, q_off + q_len) : r_len0);
  const int r_start2 = work2[blockIdx.x * 2];
  const int r_len2 = max(work2[blockIdx.x * 2 + 1], 0);
  const int n0 = (kend0 + KT - 1) / KT;
  const int ntiles = n0 + (r_len2 + KT - 1) / KT;
  int t_lo = 0, t_hi = ntiles;
  if constexpr (SPL) {
    const int per = (ntiles + (int)gridDim.z - 1) / (int)gridDim.z;
    t_lo = min(ntiles, (int)blockIdx.z * per);
    t_hi = min(ntiles, t_lo + per);
  }

  const int fr = lane & 15, grp = lane >> 4;
  // LDS-DMA of tile t into ring slot b: this wave's chunks are w * NI + i of each operand; lane L
  // of a chunk lands at row chunk * RPI + L / CH, physical 16-byte column L % CH, so it reads the
  // logical column that the swizzled read expects there
  const int drow = lane / CH, dpc = lane % CH;
  auto issue = [&](int t, int b) {
    const bool r2 = t >= n0;
    const int k0 = (r2 ? t - n0 : t) * KT;
    const int klen = r2 ? r_len2 : kend0;
    const half_t* src = kv0 + (size_t)(r2 ? r_start2 : r_start0) * ld_kv0;
    char* Kd = smem + b * 2 * TB;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int c = w * NI + i;
      const int row = c * RPI + drow;
      const half_t* rp = src + (size_t)min(k0 + row, klen - 1) * ld_kv0;
      glds16(rp + g * HD + ((dpc ^ (row & Lds<HD>::KM)) << 3), Kd + c * 1024);
      glds16(rp + (nkv + g) * HD + ((dpc ^ ((row & Lds<HD>::VM) << 1)) << 3), Kd + TB + c * 1024);
    }
  };
  const int P = hpg * q_len;                // packed rows of the item

  for (int p0 = 0; p0 < P; p0 += NW * 16) {
    // this lane's packed row (rows past P repeat the last one: finite, never stored)
    const int pw0 = p0 + w * 16;
    const bool live = pw0 < P;              // wave-uniform: waves past the item's rows only load
    const int p = min(pw0 + fr, P - 1);
    const int hh = p / q_len, r = p - hh * q_len;
    const int qr = q_start + r;
    half8 qf[NS];
    {
      const half_t* qp = qkv + (size_t)qr * ld_qkv + (g * hpg + hh) * HD + grp * 8;
#pragma unroll
      for (int s = 0; s < NS; ++s) qf[s] = *(const half8*)(qp + s * 32);
    }
    const int hi0 = r_causal0 ? min(kend0, q_off + r + 1) : kend0;     // range 0: keys [0, hi0)
    const int lo2 = r2win[2 * qr] - r_start2;                          // range 2: keys [lo2, hi2)
    const int hi2 = min(r2win[2 * qr + 1] - r_start2, r_len2);
    // (lo2_, hi2_ below: the same values, pinned before the DMAs)
    floatx4 o[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) o[u] = floatx4{0.f, 0.f, 0.f, 0.f};
    float m_run = -1e30f, l_run = 0.f;

    // the loads above retire before the tile DMAs are counted (the operands pin their uses here,
    // so the compiler's own wait for them does not land behind the DMAs and drain the ring)
    int lo2_ = lo2, hi2_ = hi2;
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(lo2_), "+v"(hi2_)::"memory");
#pragma unroll
    for (int s = 0; s < NS; ++s) asm volatile("" : "+v"(qf[s]));
#pragma unroll
    for (int i = 0; i < NB - 1; ++i)
      if (t_lo + i < t_hi) issue(t_lo + i, i);
    for (int t = t_lo; t < t_hi; ++t) {
      const int b = (t - t_lo) % NB;
      // tile t landed: the tiles issued after it may stay in flight
      const int after = min(NB - 2, t_hi - 1 - t);
      if (after >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * NI) : "memory");
      else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NI) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // tile t landed (every wave's part; no wave still reads tile t-1, whose MFMAs consumed their
      // operands): a raw barrier — __syncthreads' fence would wait for the DMAs still in flight
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t + NB - 1 < t_hi) issue(t + NB - 1, (t + NB - 1 - t_lo) % NB);
      if (!live) continue;
      const char* Ks = smem + b * 2 * TB;
      const char* Vs = Ks + TB;
      const bool r2 = t >= n0;
      const int k0 = (r2 ? t - n0 : t) * KT;
      // ---- S^T = K Q^T
      floatx4 sc[4];
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        sc[tt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < NS; ++s)
          sc[tt] = mfma16x16x32(*(const half8*)(Ks + Lds<HD>::k_off(tt * 16 + fr, s * 4 + grp)), qf[s], sc[tt]);
      }
      // ---- visibility: range 0 tiles inside every row's keys take the unmasked path
      if (r2 || r_causal0 || k0 + KT > kend0) {
        asm volatile("" ::: "memory");
        const int lo_rel = (r2 ? lo2_ : 0) - k0 - grp * 4;
        const int hi_rel = (r2 ? hi2_ : hi0) - k0 - grp * 4;             // exclusive
#pragma unroll
        for (int tt = 0; tt < 4; ++tt)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (tt * 16 + i >= hi_rel || tt * 16 + i < lo_rel) sc[tt][i] = -INFINITY;
      }
      // ---- online softmax (deferred rescale as in attn_fwd)
      float ma = vmax3(sc[0][0], sc[0][1], sc[0][2]);
      float mb = vmax3(sc[2][0], sc[2][1], sc[2][2]);
      ma = vmax3(ma, sc[0][3], sc[1][0]);
      mb = vmax3(mb, sc[2][3], sc[3][0]);
      ma = vmax3(ma, sc[1][1], sc[1][2]);
      mb = vmax3(mb, sc[3][1], sc[3][2]);
      const float mx = max_xor16_32(vmax3(ma, sc[1][3], vmax(mb, sc[3][3])));
      if (!__all((mx - m_run) * scale_log2 <= DEFER_LOG2)) {
        const float m_new = (mx - m_run) * scale_log2 > DEFER_LOG2 ? mx : m_run;   // per row (attn_fwd)
        const float alpha = fast_exp2((m_run - m_new) * scale_log2);
        l_run *= alpha;
#pragma unroll
        for (int u = 0; u < NU; ++u) o[u] *= alpha;
        m_run = m_new;
      }
      const float mc = m_run * scale_log2;
      float psum = 0.f;
      unsigned pw[8];
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        float pr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pr[i] = fast_exp2(__builtin_fmaf(sc[tt][i], scale_log2, -mc));
          psum += pr[i];
        }
        pw[tt * 2] = pack_h2(pr[0], pr[1]);
        pw[tt * 2 + 1] = pack_h2(pr[2], pr[3]);
      }
      l_run += psum;
      // ---- O^T += V^T P^T; P^T element (tt & 1) * 4 + i of k-step tt >> 1 = key 16 tt + 4 grp + i.
      // V^T by inline-asm transposed reads in groups of 4 subtiles (reads of the next group in
      // flight under the MFMAs of this one): the builtin's reads make the compiler drain every
      // outstanding LDS-DMA first (vmcnt(0)), i.e. the whole tile ring
      const int q4 = (lane & 15) >> 2, p4 = lane & 3;
      constexpr int UG = 4;                 // subtiles per read group (NU = 4 or 8)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const half8 pf = __builtin_bit_cast(half8, u32x4{pw[ks * 4], pw[ks * 4 + 1], pw[ks * 4 + 2], pw[ks * 4 + 3]});
        const int row_a = ks * 32 + grp * 4 + q4;
        half4 va[NU], vb[NU];
        auto read_group = [&](int u0) {
#pragma unroll
          for (int u = u0; u < u0 + UG; ++u) {
            const int ch = u * 2 + (p4 >> 1);
            va[u] = lds_tr16_async(Vs + Lds<HD>::v_off(row_a, ch) + (p4 & 1) * 8);
            vb[u] = lds_tr16_async(Vs + Lds<HD>::v_off(row_a + 16, ch) + (p4 & 1) * 8);
          }
        };
        read_group(0);
#pragma unroll
        for (int u0 = 0; u0 < NU; u0 += UG) {
          lds_wait4(va[u0], va[u0 + 1], va[u0 + 2], va[u0 + 3], vb[u0], vb[u0 + 1], vb[u0 + 2], vb[u0 + 3]);
          if (u0 + UG < NU) read_group(u0 + UG);
#pragma unroll
          for (int u = u0; u < u0 + UG; ++u) {
            const half8 vf = {va[u][0], va[u][1], va[u][2], va[u][3], vb[u][0], vb[u][1], vb[u][2], vb[u][3]};
            o[u] = mfma16x16x32(vf, pf, o[u]);
          }
        }
      }
    }
    // ---- normalise and store this wave's rows (split: the slice's fp32 partials)
    if (live) {
      float l = l_run;
      l += __shfl_xor(l, 16, 64);
      l += __shfl_xor(l, 32, 64);
      if (pw0 + fr < P) {
        const int h = g * hpg + hh;
        if constexpr (SPL) {
          float* pp = part + ((size_t)(qr * (int)gridDim.z + (int)blockIdx.z) * nh + h) * (HD + 2);
#pragma unroll
          for (int u = 0; u < NU; ++u) *(floatx4*)(pp + u * 16 + grp * 4) = o[u];
          if (grp == 0) *(float2_*)(pp + HD) = float2_{m_run * scale_log2, l};
        } else {
          const float inv = 1.f / l;
          half_t* op = out + (size_t)qr * ld_out + h * HD + grp * 4;
#pragma unroll
          for (int u = 0; u < NU; ++u) {
            half4 v;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = (half_t)(o[u][i] * inv);
            *(half4*)(op + u * 16) = v;
          }
        }
      }
    }
    __syncthreads();                        // the ring is the next pass's
  }
}

// tile ring depth 3 (two tiles in flight); 4 measured slower at the 70B decode shape:
// 46.3 vs 42.7 us per launch, HBM-resident caches (profiles/r5_gen/attn_decode_ring.log)
constexpr int DECODE_RING = 3;

template <int HD>
int launch_decode(dim3 grid, int ns, hipStream_t st, const half_t* qkv, half_t* out, const int* work, int nh, int nkv,
                  int ld_qkv, int ld_out, float scale_log2, const half_t* kv0, int ld_kv0, const int* work2,
                  const int* r2win, float* part) {
  if (ns > 1) {
    hipLaunchKernelGGL((attn_decode<HD, true, DECODE_RING>), dim3(grid.x, grid.y, ns), dim3(256), 0, st, qkv, out,
                       work, nh, nkv, ld_qkv, ld_out, scale_log2, kv0, ld_kv0, work2, r2win, part);
    FLS_CHECK_LAUNCH();
    hipLaunchKernelGGL((attn_split_combine<HD>), dim3(grid.x, nh), dim3(HD), 0, st, part, out, work, nh, ld_out, ns);
  } else {
    hipLaunchKernelGGL((attn_decode<HD, false, DECODE_RING>), grid, dim3(256), 0, st, qkv, out, work, nh, nkv, ld_qkv,
                       ld_out, scale_log2, kv0, ld_kv0, work2, r2win, nullptr);
  }
  FLS_CHECK_LAUNCH();
  return 0;
}

template <int HD, int WPH, bool R2>
int launch(int hpb, dim3 grid, hipStream_t st, const half_t* qkv, half_t* out, const int* work, const int* seg_lo,
           int nh, int nkv, int ld_qkv, int ld_out, float scale_log2, const half_t* kv0, int ld_kv0,
           const int* work2, const int* r2win, float* part, int ns) {
  if constexpr (R2 && HD != 96) {
    if (ns > 1) {
      const dim3 g3(grid.x, grid.y, ns);
#define FLS_ATTN_LAUNCH_SPL(HPB_)                                                                              \
  hipLaunchKernelGGL((attn_fwd<HD, HPB_, WPH, true, true>), g3, dim3(64 * WPH * HPB_), 0, st, qkv, out, work, seg_lo, \
                     nh, nkv, ld_qkv, ld_out, scale_log2, kv0, ld_kv0, work2, r2win, part)
      if constexpr (WPH == 1) {
        if (hpb == 8) FLS_ATTN_LAUNCH_SPL(8);
        else FLS_ATTN_LAUNCH_SPL(4);
      } else if constexpr (WPH == 2) {
        if (hpb == 4) FLS_ATTN_LAUNCH_SPL(4);
        else if (hpb == 2) FLS_ATTN_LAUNCH_SPL(2);
        else FLS_ATTN_LAUNCH_SPL(1);
      } else {
        if (hpb == 2) FLS_ATTN_LAUNCH_SPL(2);
        else FLS_ATTN_LAUNCH_SPL(1);
      }
#undef FLS_ATTN_LAUNCH_SPL
      FLS_CHECK_LAUNCH();
      hipLaunchKernelGGL((attn_split_combine<HD>), dim3(grid.x, nh), dim3(HD), 0, st, part, out, work, nh, ld_out, ns);
      FLS_CHECK_LAUNCH();
      return 0;
    }
  }
#define FLS_ATTN_LAUNCH(HPB_)                                                                                  \
  hipLaunchKernelGGL((attn_fwd<HD, HPB_, WPH, R2>), grid, dim3(64 * WPH * HPB_), 0, st, qkv, out, work, seg_lo, nh, \
                     nkv, ld_qkv, ld_out, scale_log2, kv0, ld_kv0, work2, r2win, nullptr)
  if constexpr (HD == 96) {
    FLS_ATTN_LAUNCH(1);                     // 12 chunks per row: one head per block divides the tile
  } else if constexpr (WPH == 1) {          // 4 or 8 heads (dispatch)
    if (hpb == 8) FLS_ATTN_LAUNCH(8);
    else FLS_ATTN_LAUNCH(4);
  } else if constexpr (WPH == 2) {
    if (hpb == 4) FLS_ATTN_LAUNCH(4);
    else if (hpb == 2) FLS_ATTN_LAUNCH(2);
    else FLS_ATTN_LAUNCH(1);
  } else {
    if (hpb == 2) FLS_ATTN_LAUNCH(2);
    else FLS_ATTN_LAUNCH(1);
  }

#undef FLS_ATTN_LAUNCH
  FLS_CHECK_LAUNCH();
  return 0;
}

// persistent attn_fwd (attn_fwd_pers): grid = the kernel's resident blocks per CU x the CUs, rounded
// down to a multiple of the head groups (a block then keeps one head group), at most the units
template <int HD, int HPB, int WPH>
void launch_pers_hpb(int n_items, int nh, hipStream_t st, const half_t* qkv, half_t* out, const int* work,
                     const int* seg_lo, int nkv, int ld_qkv, int ld_out, float scale_log2, const half_t* kv0,
                     int ld_kv0) {
  static int slots = 0;
  if (!slots) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)attn_fwd_pers<HD, HPB, WPH>,
                                                        64 * WPH * HPB, 0);
    slots = max(1, cus) * max(1, per);
  }
  const int n_hg = nh / HPB;
  const long units = (long)n_items * n_hg;
  int G = slots >= n_hg ? slots / n_hg * n_hg : slots;
  if (units < G) G = (int)units;
  hipLaunchKernelGGL((attn_fwd_pers<HD, HPB, WPH>), dim3(G), dim3(64 * WPH * HPB), 0, st, qkv, out, work, seg_lo,
                     nh, nkv, ld_qkv, ld_out, scale_log2, kv0, ld_kv0, n_items);
}

template <int HD, int WPH>
int launch_pers(int hpb, int n_items, hipStream_t st, const half_t* qkv, half_t* out, const int* work,
                const int* seg_lo, int nh, int nkv, int ld_qkv, int ld_out, float scale_log2, const half_t* kv0,
                int ld_kv0) {
#define FLS_ATTN_PERS(HPB_) \
  launch_pers_hpb<HD, HPB_, WPH>(n_items, nh, st, qkv, out, work, seg_lo, nkv, ld_qkv, ld_out, scale_log2, kv0, ld_kv0)
  if constexpr (WPH == 2) {
    if (hpb == 4) FLS_ATTN_PERS(4);
    else if (hpb == 2) FLS_ATTN_PERS(2);
    else FLS_ATTN_PERS(1);
  } else {
    if (hpb == 2) FLS_ATTN_PERS(2);
    else FLS_ATTN_PERS(1);
  }
#undef FLS_ATTN_PERS
  FLS_CHECK_LAUNCH();
  return 0;
}

int g_pers = 1;  // persistent full-pass kernel (attn_fwd_pers) on (1, default) or off (0; tests / A-B)
int g_hpb = 0;   // heads per block override (0: by group size; tests / A-B)
int g_split = 0; // split-KV slices of the range-2 kernel: 0 = by grid size, 1 = off, n = n (tests / A-B)

}  // namespace

// heads of one KV group per block: 0 = by group size (default), else 1 / 2 / 4 (A/B)
extern "C" int fls_attention_set_hpb(int hpb) {
  const int old = g_hpb;
  g_hpb = hpb;
  return old;
}

// persistent full-pass kernel on (1, default) / off (0: one block per work item x head group)
extern "C" int fls_attention_set_persistent(int on) {
  const int old = g_pers;
  g_pers = on ? 1 : 0;
  return old;
}

extern "C" int fls_attention_set_split(int ns) {
  const int old = g_split;
  g_split = ns;
  return old;
}

namespace {
template <bool R2>
int dispatch(const void* qkv, void* out, const int* work, int n_items, int n_q_heads, int n_kv_heads, int head_dim,
             int ld_qkv, int ld_out, float scale, const void* kv0, int ld_kv0, const int* seg_lo, int q_block,
             const int* work2, const int* r2win, void* ws, unsigned long long ws_bytes, int n_rows,
             fls_stream_t s) {
  if (n_q_heads % n_kv_heads) return -2;
  if (head_dim != 64 && head_dim != 96 && head_dim != 128) return -3;
  // q_block 32 (one wave per head): range-2 items of at most 32 rows (generation steps);
  // q_block 8: range-2 items of at most 8 rows, packed-GQA decode kernel
  if (q_block != 64 && q_block != 128 && !(R2 && (q_block == 32 || q_block == 8))) return -5;
  const float scale_log2 = scale * 1.4426950408889634f;
  auto st = (hipStream_t)s;
  const int group = n_q_heads / n_kv_heads;
  if constexpr (R2) {
    if (q_block == 8 && head_dim != 96) {
      // one block per (item, KV group), 4 waves; split the key tiles over blocks only when the
      // grid leaves CUs idle (one block per CU at this kernel's register use)
      const dim3 grid(n_items, n_kv_heads);
      const long blocks = (long)grid.x * grid.y;
      int ns = 1;
      if (ws && n_rows > 0) {
        ns = g_split > 0 ? g_split : (blocks >= 192 ? 1 : (int)min(8L, (256 + blocks - 1) / blocks));
        const unsigned long long per = (unsigned long long)n_rows * n_q_heads * (head_dim + 2) * 4ull;
        while (ns > 1 && per * ns > ws_bytes) --ns;
      }
      auto q = (const half_t*)qkv;
      auto o = (half_t*)out;
      auto k0 = (const half_t*)kv0;
      return head_dim == 128 ? launch_decode<128>(grid, ns, st, q, o, work, n_q_heads, n_kv_heads, ld_qkv, ld_out,
                                                  scale_log2, k0, ld_kv0, work2, r2win, (float*)ws)
                             : launch_decode<64>(grid, ns, st, q, o, work, n_q_heads, n_kv_heads, ld_qkv, ld_out,
                                                 scale_log2, k0, ld_kv0, work2, r2win, (float*)ws);
    }
  }
  if (q_block == 8) q_block = 32;           // hd 96 (or the non-range-2 kernel): the per-head layout
  // heads of one KV group per block share every staged K/V tile: up to 4 (64-row items) or 2
  // (128-row items, 4 waves per head) as the group allows, else 1 (multi-head attention)
  // (32-row items: up to 8, a whole 70B KV group, so every prompt's prefix K/V is read once per
  // layer; 8 heads x 2 waves = 1024 threads measured 4x slower (profiles/r3_attn): not built)
  // one wave per head pays only with several heads per block (a 64-thread block of 16 staging
  // chunks per lane and 2 waves per CU would not): small groups keep the 2-wave layout
  if (q_block == 32 && (group % 4 || head_dim == 96)) q_block = 64;
  const int hpb_max = q_block == 32 ? 8 : (q_block == 64 ? 4 : 2);
  int hpb = 1;
  while (hpb * 2 <= hpb_max && group % (hpb * 2) == 0) hpb *= 2;
  if (g_hpb > 0 && group % g_hpb == 0 && g_hpb <= hpb_max && (q_block != 32 || g_hpb >= 4)) hpb = g_hpb;
  if (head_dim == 96) hpb = 1;              // Phi-3-mini geometry (multi-head attention anyway)
  const dim3 grid(n_items, n_q_heads / hpb);
  // split-KV (range-2 kernel) only when the grid leaves CUs idle (a long prompt or two decoding
  // alone: one block per (item, 4 heads)); at 2 blocks per CU, the occupancy limit, the slices just
  // queue behind each other and the combine costs extra: 70B, 32 prompts x 5 suffixes (512 blocks),
  // 0.058 s per generation step unsplit vs 0.061-0.063 s split in 4 (profiles/r3_splitkv)
  int ns = 1;
  if (R2 && head_dim != 96 && ws && n_rows > 0) {
    const long blocks = (long)grid.x * grid.y;
    ns = g_split > 0 ? g_split : (blocks >= 256 ? 1 : (int)min(8L, (512 + blocks - 1) / blocks));
    const unsigned long long per = (unsigned long long)n_rows * n_q_heads * (head_dim + 2) * 4ull;
    while (ns > 1 && per * ns > ws_bytes) --ns;
  }
  float* part = (float*)ws;
  auto q = (const half_t*)qkv;
  auto o = (half_t*)out;
  auto k0 = (const half_t*)kv0;
  if constexpr (!R2) {
    if (g_pers && head_dim != 96 && q_block != 32)
      return q_block == 64 ? (head_dim == 128 ? launch_pers<128, 2>(hpb, n_items, st, q, o, work, seg_lo, n_q_heads,
                                                                    n_kv_heads, ld_qkv, ld_out, scale_log2, k0, ld_kv0)
                                              : launch_pers<64, 2>(hpb, n_items, st, q, o, work, seg_lo, n_q_heads,
                                                                   n_kv_heads, ld_qkv, ld_out, scale_log2, k0, ld_kv0))
                           : (head_dim == 128 ? launch_pers<128, 4>(hpb, n_items, st, q, o, work, seg_lo, n_q_heads,
                                                                    n_kv_heads, ld_qkv, ld_out, scale_log2, k0, ld_kv0)
                                              : launch_pers<64, 4>(hpb, n_items, st, q, o, work, seg_lo, n_q_heads,
                                                                   n_kv_heads, ld_qkv, ld_out, scale_log2, k0, ld_kv0));
  }
  if constexpr (R2) {
    if (q_block == 32)                      // head_dim 64 / 128 here (96 fell back above)
      return head_dim == 128 ? launch<128, 1, true>(hpb, grid, st, q, o, work, seg_lo, n_q_heads, n_kv_heads, ld_qkv,
                                                    ld_out, scale_log2, k0, ld_kv0, work2, r2win, part, ns)
                             : launch<64, 1, true>(hpb, grid, st, q, o, work, seg_lo, n_q_heads, n_kv_heads, ld_qkv,
                                                   ld_out, scale_log2, k0, ld_kv0, work2, r2win, part, ns);
  }
  if (head_dim == 96)
    return q_block == 64 ? launch<96, 2, R2>(hpb, grid, st, q, o, work, seg_lo, n_q_heads, n_kv_heads, ld_qkv, ld_out,
                                         scale_log2, k0, ld_kv0, work2, r2win, part, ns)
                         : launch<96, 4, R2>(hpb, grid, st, q, o, work, seg_lo, n_q_heads, n_kv_heads, ld_qkv, ld_out,
                                         scale_log2, k0, ld_kv0, work2, r2win, part, ns);
  if (q_block == 64)
    return head_dim == 128 ? launch<128, 2, R2>(hpb, grid, st, q, o, work, seg_lo, n_q_heads, n_kv_heads, ld_qkv, ld_out,
                                            scale_log2, k0, ld_kv0, work2, r2win, part, ns)
                           : launch<64, 2, R2>(hpb, grid, st, q, o, work, seg_lo, n_q_heads, n_kv_heads, ld_qkv, ld_out,
                                           scale_log2, k0, ld_kv0, work2, r2win, part, ns);
  return head_dim == 128 ? launch<128, 4, R2>(hpb, grid, st, q, o, work, seg_lo, n_q_heads, n_kv_heads, ld_qkv, ld_out,
                                          scale_log2, k0, ld_kv0, work2, r2win, part, ns)
                         : launch<64, 4, R2>(hpb, grid, st, q, o, work, seg_lo, n_q_heads, n_kv_heads, ld_qkv, ld_out,
                                         scale_log2, k0, ld_kv0, work2, r2win, part, ns);
}
}  // namespace

extern "C" int fls_attention(const void* qkv, void* out, const int* work, int n_items, int n_q_heads,
                             int n_kv_heads, int head_dim, int ld_qkv, int ld_out, float scale, const void* kv0,
                             int ld_kv0, const int* seg_lo, int q_block, const int* work2, const int* r2win,
                             void* ws, unsigned long long ws_bytes, int n_rows, fls_stream_t s) {
  if (n_items <= 0) return 0;
  if (work2 && (!kv0 || !r2win)) return -6;   // range 2 indexes the K/V cache, per-row windows
  return work2 ? dispatch<true>(qkv, out, work, n_items, n_q_heads, n_kv_heads, head_dim, ld_qkv, ld_out, scale, kv0,
                                ld_kv0, seg_lo, q_block, work2, r2win, ws, ws_bytes, n_rows, s)
               : dispatch<false>(qkv, out, work, n_items, n_q_heads, n_kv_heads, head_dim, ld_qkv, ld_out, scale, kv0,
                                 ld_kv0, seg_lo, q_block, nullptr, nullptr, nullptr, 0, 0, s);
}
