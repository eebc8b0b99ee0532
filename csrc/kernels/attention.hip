// Shared-prefix / varlen flash attention forward on gfx950 (MI355X).
//
// Replaces the reference's eager attention (HF LlamaAttention via
// utils.py:272-279): prefix K/V expanded to every suffix, concatenated, then
// repeat_kv'd to every query head — materialised n_s * (nh/nkv) times — and a
// [1, nh, Lp, Lp] fp32 probability matrix.
//
// Here K/V are read IN PLACE from the packed QKV activation: a work item is
// a block of <= 64 query rows of one segment plus up to two key ranges
//   range 0: the prompt's prefix (bidirectional, or causal for prefix queries
//            in --prefix_attention causal),
//   range 1: the suffix's own tokens, causal (key j visible to query i iff j <= i),
// so every suffix of a prompt reads the single shared prefix K/V, GQA-native
// (query head h uses kv head h / (nh/nkv)).
//
// Structure (4 waves x 16 query rows; K/V tiles of 64 keys in LDS):
//   * S^T = K . Q^T with v_mfma_f32_16x16x32_f16 (A = K fragment from LDS,
//     B = Q fragment in registers), so each lane owns ONE query row's scores:
//     the online-softmax max/sum needs only 2 cross-lane xor steps and the
//     P fragment for the next MFMA is lane-local (no LDS round trip);
//   * O^T += V^T . P^T: the V^T operand comes from ds_read_b64_tr_b16
//     (hardware transpose read, guide T10) of a row-major, XOR-swizzled V
//     tile; O^T keeps the query on the lane too, so rescaling by
//     exp2(m_old - m_new) is lane-local;
//   * K tile XOR-swizzled per 16-byte chunk for conflict-free ds_read_b128.
#include "common.h"
#include "fls.h"

namespace {

constexpr int KT = 64;       // keys per tile
constexpr int QB = 64;       // query rows per work item (4 waves x 16)

template <int HD>
struct Lds {
  static constexpr int ROW = HD * 2;            // bytes per row
  static constexpr int NCH = HD / 8;            // 16-byte chunks per row
  // K: ds_read_b128 row reads -> chunk ^ (row & (NCH-1))
  __device__ static int k_off(int row, int ch) { return row * ROW + ((ch ^ (row & (NCH - 1))) << 4); }
  // V: ds_read_b64_tr_b16 -> chunk ^ ((row & (NCH/2-1)) << 1)
  __device__ static int v_off(int row, int ch) { return row * ROW + ((ch ^ ((row & (NCH / 2 - 1)) << 1)) << 4); }
};

// HPB query heads of the same KV group per block (GQA): waves 4*j .. 4*j+3
// serve head h0 + j, so every K/V tile staged in LDS feeds 4*HPB waves.
template <int HD, int HPB>
__global__ __launch_bounds__(256 * HPB) void attn_fwd(const half_t* __restrict__ qkv, half_t* __restrict__ out,
                                                    const int* __restrict__ work, int nh, int nkv, int ld_qkv,
                                                    int ld_out, float scale_log2, const half_t* __restrict__ kv0,
                                                    int ld_kv0) {
  constexpr int NS = HD / 32;     // k-steps of the QK^T product
  constexpr int NU = HD / 16;     // 16-wide d subtiles of O
  __shared__ __attribute__((aligned(16))) char smem[2 * KT * HD * 2];
  char* Ks = smem;
  char* Vs = smem + KT * HD * 2;

  constexpr int NT_ = 256 * HPB;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = (tid >> 6) & 3;          // row group inside the 64-row item
  const int h = blockIdx.y * HPB + (tid >> 8);
  const int g = h / (nh / nkv);

  const int* wi = work + blockIdx.x * 8;
  const int q_start = wi[0], q_len = wi[1], q_off = wi[2];
  if (q_len <= 0) return;                   // padding item (bucketed graph replays); block-uniform
  const int r_start[2] = {wi[3], wi[6]};
  const int r_len[2] = {wi[4], wi[7]};
  const int r_causal[2] = {wi[5], 1};

  const int fr = lane & 15, grp = lane >> 4;
  const int q_col = h * HD;
  const int k_col = nh * HD + g * HD;
  const int v_col = (nh + nkv) * HD + g * HD;

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[row fr][32s + 8grp .. +8]
  const int qrow = wave * 16 + fr;
  const int qrow_c = min(qrow, q_len - 1);
  half8 qf[NS];
  {
    const half_t* qp = qkv + (size_t)(q_start + qrow_c) * ld_qkv + q_col + grp * 8;
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[s] = *(const half8*)(qp + s * 32);
  }
  const int qi = q_off + qrow;   // query index within its segment (causal compare)

  floatx4 o[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) o[u] = floatx4{0.f, 0.f, 0.f, 0.f};
  float m_run = -1e30f;
  float l_run = 0.f;

  for (int rg = 0; rg < 2; ++rg) {
    const int klen = r_len[rg];
    if (klen <= 0) continue;
    const int kbase = r_start[rg];
    const bool causal = r_causal[rg] != 0;
    // range 0 may live in the prefix K/V cache ([P, 2 * nkv * HD], K then V)
    const bool from_cache = rg == 0 && kv0 != nullptr;
    const half_t* kvb = from_cache ? kv0 : qkv;
    const int ldk = from_cache ? ld_kv0 : ld_qkv;
    const int kc = from_cache ? g * HD : k_col;
    const int vc = from_cache ? (nkv + g) * HD : v_col;
    // keys needed by the last valid query of this block
    const int kend = causal ? min(klen, q_off + q_len) : klen;
    for (int k0 = 0; k0 < kend; k0 += KT) {
      __syncthreads();
      // ---- stage K and V tiles (64 rows x HD) into LDS, 16 B per thread-chunk
      constexpr int CHUNKS = KT * HD / 8;
#pragma unroll
      for (int c = tid; c < CHUNKS; c += NT_) {
        const int row = c / (HD / 8), ch = c % (HD / 8);
        const int key = min(k0 + row, klen - 1);
        const half_t* src = kvb + (size_t)(kbase + key) * ldk;
        const half8 kv = *(const half8*)(src + kc + ch * 8);
        const half8 vv = *(const half8*)(src + vc + ch * 8);
        *(half8*)(Ks + Lds<HD>::k_off(row, ch)) = kv;
        *(half8*)(Vs + Lds<HD>::v_off(row, ch)) = vv;
      }
      __syncthreads();

      // ---- S^T tile: 4 subtiles of 16 keys; lane holds keys 16t + 4grp + r of query fr
      floatx4 sc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        sc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
        const int krow = t * 16 + fr;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const half8 kf = *(const half8*)(Ks + Lds<HD>::k_off(krow, s * 4 + grp));
          sc[t] = mfma16x16x32(kf, qf[s], sc[t]);
        }
      }
      // ---- scale, mask, online softmax (query = lane's fr row)
      float mx = -INFINITY;
      // key k0 + 16t + 4grp + r is visible iff 16t + r <= rel (one compare per score)
      const int rel = (causal ? min(klen - 1, qi) : klen - 1) - k0 - grp * 4;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = (t * 16 + r <= rel) ? sc[t][r] * scale_log2 : -INFINITY;
          sc[t][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx);
      // rescale only when some row's max grew (alpha == 1 exactly otherwise)
      if (!__all(m_new == m_run)) {
        const float alpha = fast_exp2(m_run - m_new);
        l_run *= alpha;
#pragma unroll
        for (int u = 0; u < NU; ++u) o[u] *= alpha;
      }
      m_run = m_new;
      float psum = 0.f;
      half8 pf[2];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = fast_exp2(sc[t][r] - m_new);
          psum += p;
          pf[t >> 1][(t & 1) * 4 + r] = (half_t)p;
        }
      l_run += psum;

      // ---- O^T += V^T P^T ; V^T fragment via two transposed 4x16 reads
      const int q4 = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int row_a = ks * 32 + grp * 4 + q4;
        const int row_b = row_a + 16;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int ch = u * 2 + (p4 >> 1);
          const half4 va = ds_read_tr16(Vs + Lds<HD>::v_off(row_a, ch) + (p4 & 1) * 8);
          const half4 vb = ds_read_tr16(Vs + Lds<HD>::v_off(row_b, ch) + (p4 & 1) * 8);
          const half8 vf = {va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]};
          o[u] = mfma16x16x32(vf, pf[ks], o[u]);
        }
      }
    }
  }
  // ---- normalise and store: lane holds O[q = fr][d = 16u + 4grp + r]
  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);
  if (qrow < q_len) {
    const float inv = 1.f / l_run;
    half_t* op = out + (size_t)(q_start + qrow) * ld_out + h * HD + grp * 4;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      half4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (half_t)(o[u][r] * inv);
      *(half4*)(op + u * 16) = v;
    }
  }
}

// ------------------------------------------------------------------- v2
// LDS-read intensity is what bounds attn_fwd: every wave re-reads the whole
// 64-key K and V tile (32 KB) from LDS for only 16 query rows (32 MFMAs), so
// the LDS pipe needs ~2x the MFMA time.  v2 gives each wave 32 query rows
// (two 16-row groups sharing every K / V^T fragment it reads: 64 MFMAs per
// 32 KB) with 2 waves per query head and HPB heads of one KV group per block,
// and overlaps the global->LDS staging with compute: tile t+1's K/V rows are
// loaded into registers before tile t's MFMAs and written to LDS after the
// barrier that retires tile t's reads (guide T14, write-after-barrier).
// The key tiles of both ranges (prefix, own suffix) form one flat sequence so
// the prefetch crosses the range boundary.  DB = true (variant 3, default)
// double-buffers the LDS tile: tile t+1 is written into the other buffer right
// after tile t's MFMAs and tile t+2's loads are issued, one barrier per tile.
// Masking is one integer compare per score against a per-lane visibility
// bound, and the O / l rescale is skipped when no row's running max grew
// (alpha would be exactly 1).
// Measured (profiles/r1_attention): 1024-token prefix + 5x64 suffixes, 70B
// heads: v1 598 -> v3 727 TFLOP/s; 4096-token prefix: 683 -> 870.
// WPH: waves per query head (32 query rows each) = rows per work item / 32.  WPH = 4 (128-row
// items) serves multi-head attention, where no other head shares the K/V tile: 4 waves read it.
template <int HD, int HPB, bool DB, int WPH = 2>
__global__ __launch_bounds__(64 * WPH * HPB, 2) void attn_fwd_v2(const half_t* __restrict__ qkv, half_t* __restrict__ out,
                                                       const int* __restrict__ work, int nh, int nkv, int ld_qkv,
                                                       int ld_out, float scale_log2,
                                                       const half_t* __restrict__ kv0, int ld_kv0) {
  constexpr int NT_ = 64 * WPH * HPB;
  constexpr int NS = HD / 32;               // k-steps of QK^T
  constexpr int NU = HD / 16;               // 16-wide d subtiles of O
  constexpr int CH = HD / 8;                // 16-byte chunks per K/V row
  constexpr int PER = KT * CH / NT_;        // chunks per thread per operand
  static_assert(PER >= 1 && (KT * CH) % NT_ == 0, "tile / block mismatch");
  constexpr int TILE_BYTES = 2 * KT * HD * 2;         // K + V
  __shared__ __attribute__((aligned(16))) char smem[(DB ? 2 : 1) * TILE_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int h = blockIdx.y * HPB + wave / WPH;
  const int g = h / (nh / nkv);             // same for every head of the block (HPB | group)
  const int rbase = (wave % WPH) * 32;      // this wave's first query row of the item

  const int* wi = work + blockIdx.x * 8;
  const int q_start = wi[0], q_len = wi[1], q_off = wi[2];
  if (q_len <= 0) return;                   // padding item (bucketed graph replays); block-uniform
  const int r_start0 = wi[3], r_len0 = wi[4], r_causal0 = wi[5];
  const int r_start1 = wi[6], r_len1 = wi[7];
  const int kend0 = r_len0 <= 0 ? 0 : (r_causal0 ? min(r_len0, q_off + q_len) : r_len0);
  const int kend1 = r_len1 <= 0 ? 0 : min(r_len1, q_off + q_len);
  const int n0 = (kend0 + KT - 1) / KT;
  const int ntiles = n0 + (kend1 + KT - 1) / KT;

  const int fr = lane & 15, grp = lane >> 4;
  const int q_col = h * HD;
  const int k_col = nh * HD + g * HD;
  const int v_col = (nh + nkv) * HD + g * HD;

  half8 qf[2][NS];
  int qi[2];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int qrow = rbase + qg * 16 + fr;
    const half_t* qp = qkv + (size_t)(q_start + min(qrow, q_len - 1)) * ld_qkv + q_col + grp * 8;
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[qg][s] = *(const half8*)(qp + s * 32);
    qi[qg] = q_off + qrow;
  }

  floatx4 o[2][NU];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg)
#pragma unroll
    for (int u = 0; u < NU; ++u) o[qg][u] = floatx4{0.f, 0.f, 0.f, 0.f};
  float m_run[2] = {-1e30f, -1e30f};
  float l_run[2] = {0.f, 0.f};

  half8 pk[PER], pv[PER];
  auto load_tile = [&](int t) {
    const bool r1 = t >= n0;
    const int k0 = (r1 ? t - n0 : t) * KT;
    const int klen = r1 ? r_len1 : r_len0;
    const int kb = r1 ? r_start1 : r_start0;
    // range 0 may live in the prefix K/V cache ([P, 2 * nkv * HD], K then V)
    const bool from_cache = !r1 && kv0 != nullptr;
    const half_t* kvb = from_cache ? kv0 : qkv;
    const int ldk = from_cache ? ld_kv0 : ld_qkv;
    const int kc = from_cache ? g * HD : k_col;
    const int vc = from_cache ? (nkv + g) * HD : v_col;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NT_;
      const int row = c / CH, ch = c % CH;
      const half_t* src = kvb + (size_t)(kb + min(k0 + row, klen - 1)) * ldk;
      pk[i] = *(const half8*)(src + kc + ch * 8);
      pv[i] = *(const half8*)(src + vc + ch * 8);
    }
  };
  auto store_tile = [&](int buf) {
    char* Ks = smem + buf * TILE_BYTES;
    char* Vs = Ks + KT * HD * 2;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NT_;
      const int row = c / CH, ch = c % CH;
      *(half8*)(Ks + Lds<HD>::k_off(row, ch)) = pk[i];
      *(half8*)(Vs + Lds<HD>::v_off(row, ch)) = pv[i];
    }
  };

  if (ntiles > 0) {
    load_tile(0);
    store_tile(0);
    if (DB && ntiles > 1) load_tile(1);
  }
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const bool r1 = t >= n0;
    const int k0 = (r1 ? t - n0 : t) * KT;
    const int klen = r1 ? r_len1 : r_len0;
    const bool causal = r1 || r_causal0;
    const char* Ks = smem + (DB ? (t & 1) : 0) * TILE_BYTES;
    const char* Vs = Ks + KT * HD * 2;
    if (!DB && t + 1 < ntiles) load_tile(t + 1);     // in flight under this tile's MFMAs

    // ---- S^T = K Q^T for both 16-row query groups (each K fragment read once)
    floatx4 sc[2][4];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      sc[0][tt] = floatx4{0.f, 0.f, 0.f, 0.f};
      sc[1][tt] = floatx4{0.f, 0.f, 0.f, 0.f};
      const int krow = tt * 16 + fr;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const half8 kf = *(const half8*)(Ks + Lds<HD>::k_off(krow, s * 4 + grp));
        sc[0][tt] = mfma16x16x32(kf, qf[0][s], sc[0][tt]);
        sc[1][tt] = mfma16x16x32(kf, qf[1][s], sc[1][tt]);
      }
    }
    // ---- scale, mask, online softmax per query group
    half8 pf[2][2];
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
      float mx = -INFINITY;
      const int rel = (causal ? min(klen - 1, qi[qg]) : klen - 1) - k0 - grp * 4;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = (tt * 16 + r <= rel) ? sc[qg][tt][r] * scale_log2 : -INFINITY;
          sc[qg][tt][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run[qg], mx);
      if (!__all(m_new == m_run[qg])) {
        const float alpha = fast_exp2(m_run[qg] - m_new);
        l_run[qg] *= alpha;
#pragma unroll
        for (int u = 0; u < NU; ++u) o[qg][u] *= alpha;
      }
      m_run[qg] = m_new;
      float psum = 0.f;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = fast_exp2(sc[qg][tt][r] - m_new);
          psum += p;
          pf[qg][tt >> 1][(tt & 1) * 4 + r] = (half_t)p;
        }
      l_run[qg] += psum;
    }
    // ---- O^T += V^T P^T (each V^T fragment read once for both groups)
    const int q4 = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int row_a = ks * 32 + grp * 4 + q4;
      const int row_b = row_a + 16;
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int ch = u * 2 + (p4 >> 1);
        const half4 va = ds_read_tr16(Vs + Lds<HD>::v_off(row_a, ch) + (p4 & 1) * 8);
        const half4 vb = ds_read_tr16(Vs + Lds<HD>::v_off(row_b, ch) + (p4 & 1) * 8);
        const half8 vf = {va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]};
        o[0][u] = mfma16x16x32(vf, pf[0][ks], o[0][u]);
        o[1][u] = mfma16x16x32(vf, pf[1][ks], o[1][u]);
      }
    }
    if (DB) {
      // the other buffer's last readers (tile t-1) all passed the previous barrier
      if (t + 1 < ntiles) {
        store_tile((t + 1) & 1);
        if (t + 2 < ntiles) load_tile(t + 2);   // in flight under tile t+1's MFMAs
      }
      __syncthreads();
    } else if (t + 1 < ntiles) {
      __syncthreads();          // every wave is done reading tile t
      store_tile(0);
      __syncthreads();
    }
  }
  // ---- normalise and store
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    float l = l_run[qg];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const int qrow = rbase + qg * 16 + fr;
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

int g_attn_variant = 3;
int g_attn_mha_v2 = 0;   // odd GQA groups (MHA) on the v2/v3 kernel with one head per block (A/B)

}  // namespace

extern "C" int fls_attn_set_mha_v2(int on) {
  const int old = g_attn_mha_v2;
  g_attn_mha_v2 = on ? 1 : 0;
  return old;
}

extern "C" int fls_attn_set_variant(int v) {
  if (v < 1 || v > 3) return -1;
  g_attn_variant = v;
  return 0;
}

extern "C" int fls_attention(const void* qkv, void* out, const int* work, int n_items, int n_q_heads,
                             int n_kv_heads, int head_dim, int ld_qkv, int ld_out, float scale, const void* kv0,
                             int ld_kv0, int q_block, fls_stream_t s) {
  if (n_items <= 0) return 0;
  if (n_q_heads % n_kv_heads) return -2;
  const float scale_log2 = scale * 1.4426950408889634f;
  auto st = (hipStream_t)s;
  const int group = n_q_heads / n_kv_heads;
  if (q_block > 64) {
    // 128-row work items (runtime/batch.py pack_prompts(q_block=128)): 4 waves per query head
    if (q_block > 128 || (head_dim != 64 && head_dim != 128)) return -5;
    const int hpb = group % 2 == 0 ? 2 : 1;
    dim3 grid4(n_items, n_q_heads / hpb);
#define FLS_ATTN4_LAUNCH(HD_, HPB_)                                                                       \
  hipLaunchKernelGGL((attn_fwd_v2<HD_, HPB_, true, 4>), grid4, dim3(256 * HPB_), 0, st, (const half_t*)qkv, \
                     (half_t*)out, work, n_q_heads, n_kv_heads, ld_qkv, ld_out, scale_log2,               \
                     (const half_t*)kv0, ld_kv0)
    if (head_dim == 128) {
      if (hpb == 2) FLS_ATTN4_LAUNCH(128, 2); else FLS_ATTN4_LAUNCH(128, 1);
    } else {
      if (hpb == 2) FLS_ATTN4_LAUNCH(64, 2); else FLS_ATTN4_LAUNCH(64, 1);
    }
#undef FLS_ATTN4_LAUNCH
    FLS_CHECK_LAUNCH();
    return 0;
  }
  if (g_attn_variant >= 2 && (head_dim == 64 || head_dim == 128) &&
      (group % 2 == 0 || g_attn_mha_v2)) {
    // HPB query heads of one KV group per block; odd groups (MHA: Llama-2-7B/13B) one head per block
    const int hpb = group % 4 == 0 ? 4 : (group % 2 == 0 ? 2 : 1);
    const bool db = g_attn_variant == 3;
    dim3 grid2(n_items, n_q_heads / hpb);
#define FLS_ATTN2_LAUNCH(HD_, HPB_)                                                                       \
  do {                                                                                                    \
    if (db)                                                                                               \
      hipLaunchKernelGGL((attn_fwd_v2<HD_, HPB_, true>), grid2, dim3(128 * HPB_), 0, st,                   \
                         (const half_t*)qkv, (half_t*)out, work, n_q_heads, n_kv_heads, ld_qkv, ld_out,    \
                         scale_log2, (const half_t*)kv0, ld_kv0);                                                                     \
    else                                                                                                  \
      hipLaunchKernelGGL((attn_fwd_v2<HD_, HPB_, false>), grid2, dim3(128 * HPB_), 0, st,                  \
                         (const half_t*)qkv, (half_t*)out, work, n_q_heads, n_kv_heads, ld_qkv, ld_out,    \
                         scale_log2, (const half_t*)kv0, ld_kv0);                                                                     \
  } while (0)
    if (head_dim == 128) {
      if (hpb == 4) FLS_ATTN2_LAUNCH(128, 4); else if (hpb == 2) FLS_ATTN2_LAUNCH(128, 2); else FLS_ATTN2_LAUNCH(128, 1);
    } else {
      if (hpb == 4) FLS_ATTN2_LAUNCH(64, 4); else if (hpb == 2) FLS_ATTN2_LAUNCH(64, 2); else FLS_ATTN2_LAUNCH(64, 1);
    }
#undef FLS_ATTN2_LAUNCH
    FLS_CHECK_LAUNCH();
    return 0;
  }
  const bool two = (group % 2) == 0;        // pair up query heads of one KV group
  dim3 grid(n_items, two ? n_q_heads / 2 : n_q_heads);
#define FLS_ATTN_LAUNCH(HD_, HPB_)                                                                          \
  hipLaunchKernelGGL((attn_fwd<HD_, HPB_>), grid, dim3(256 * HPB_), 0, st, (const half_t*)qkv, (half_t*)out, \
                     work, n_q_heads, n_kv_heads, ld_qkv, ld_out, scale_log2, (const half_t*)kv0, ld_kv0)
  switch (head_dim) {
    case 64:
      if (two) FLS_ATTN_LAUNCH(64, 2); else FLS_ATTN_LAUNCH(64, 1);
      break;
    case 128:
      if (two) FLS_ATTN_LAUNCH(128, 2); else FLS_ATTN_LAUNCH(128, 1);
      break;
    default:
      return -3;
  }
#undef FLS_ATTN_LAUNCH
  FLS_CHECK_LAUNCH();
  return 0;
}
