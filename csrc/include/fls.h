// flexible_llm_sharding_amd — native C ABI shared by the HIP kernel library
// (libfls_kernels.so) and the host runtime (libfls_runtime.so).
//
// Everything is exported with C linkage and raw pointers so Python binds it
// through ctypes with no PyTorch headers in the build (fast, hermetic
// builds; hipcc --offload-arch=gfx950 only).  Streams are passed as
// hipStream_t (the value of torch.cuda.Stream.cuda_stream on ROCm).
#pragma once
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* fls_stream_t;

// ----------------------------------------------------------------- runtime
int   fls_rt_version(void);
void* fls_pinned_alloc(uint64_t bytes);                  // hipHostMalloc; NULL on failure
int   fls_pinned_free(void* p);
void* fls_host_device_ptr(void* p);                    // device address of a mapped pinned block (or NULL)
int   fls_pinned_register(void* p, uint64_t bytes);      // hipHostRegister an existing range
int   fls_pinned_unregister(void* p);
int   fls_memcpy_async(void* dst, const void* src, uint64_t bytes, int kind, fls_stream_t s);
int64_t fls_pread_into(const char* path, uint64_t offset, uint64_t bytes, void* dst, int nthreads);
int64_t fls_pwrite_from(const char* path, uint64_t offset, uint64_t bytes, const void* src,
                        int nthreads, int truncate);
int   fls_gather_blocks(void* dst, const void* src, uint64_t block_bytes, const int64_t* src_block,
                        int64_t n_blocks, int nthreads);
// safetensors header index
void* fls_st_open(const char* path);
int   fls_st_count(void* h);
int   fls_st_info(void* h, int i, char* name, int name_cap, char* dtype, int dtype_cap,
                  int64_t* shape, int* ndim, uint64_t* begin, uint64_t* end);
uint64_t fls_st_data_offset(void* h);
void  fls_st_close(void* h);
int   fls_mem_info(uint64_t* free_b, uint64_t* total_b);
void* fls_device_alloc(int device, uint64_t bytes);        // hipMalloc (outside the torch allocator)
int   fls_device_free(int device, void* p);

// weight streamer: file byte ranges -> pinned chunk ring -> HBM (runtime/stream.py)
typedef struct {
  uint64_t file_off;   // byte offset in the file
  uint64_t nbytes;     // bytes in the file
  uint64_t dst_off;    // byte offset in the destination (HBM slot / host buffer)
  int32_t kind;        // 0 raw copy, 1 fp32 in the file -> fp16 (nbytes / 2 written)
  int32_t pad;
} fls_piece_t;
void*   fls_streamer_create(int device, uint64_t chunk_bytes, int n_chunks, int io_threads, int direct);
void*   fls_streamer_create_host(uint64_t chunk_bytes, int n_chunks, int io_threads, int direct, int copy_delay_us);
int     fls_streamer_sync_host(void* h);
uint64_t fls_streamer_pinned_bytes(void* h);
int64_t fls_streamer_load(void* h, const char* path, const fls_piece_t* pieces, int n, void* dst_dev,
                          fls_stream_t stream);
int64_t fls_stream_read_host(const char* path, const fls_piece_t* pieces, int n, void* dst, int io_threads);
int     fls_streamer_stats(void* h, double* read_s, double* wait_s, uint64_t* read_bytes, uint64_t* h2d_bytes,
                           int* direct_fallbacks);
void    fls_streamer_destroy(void* h);
void    fls_f32_to_f16(const float* src, uint16_t* dst, uint64_t n);

// ----------------------------------------------------------------- kernels
int fls_kernels_version(void);
// epilogue codes for fls_gemm
enum { FLS_EPI_NONE = 0, FLS_EPI_RESID = 1, FLS_EPI_SWIGLU = 2, FLS_EPI_ROPE = 3 };
// or'd into epi: row-independent arithmetic only (the v10 / v11 / mid-M tiles, else the generic
// kernel; no skinny or split-K path), so a row's result does not depend on M or on the other rows: the
// generation tie guard re-runs a subset of prompts bit-identically to the whole batch
#define FLS_GEMM_ROW_EXACT 0x100
// C[M, N'] = epi(acc), acc[m] = rscale[m] * (A[M,K] . W[N,K]^T)[m] (+ bias)  (rscale may be null:
// 1; the RMSNorm statistic of a fused norm + projection).  fp16 in / fp32 accumulate / fp16 out.
//   RESID : C = alpha * acc + R (R may alias C; alpha: Granite's residual_multiplier, else 1)
//   SWIGLU: W = [gate (N/2 rows); up (N/2 rows)]; C has N/2 columns = silu(g)*u
//   ROPE  : columns < rope_cols are rotated (HF rotate-half, natural head-dim
//           order, head_dim 64 or 128) with pos[m] and fp32 tables cos/sin
//           [maxpos, head_dim/2]
int fls_gemm(const void* A, const void* W, void* C, const void* R, int M, int N, int K,
             int lda, int ldw, int ldc, int ldr, int epi, const int* pos, const float* cos_t,
             const float* sin_t, int rope_cols, int head_dim, const void* bias, const float* rscale,
             float alpha, float* ss, int ss_ld, void* ws, uint64_t ws_bytes,
             fls_stream_t s);   // ws: device scratch for the small-M split-K path (may be null)
// ss (RESID only, may be null): ss[m * ss_ld + j] = sum of the squares of the fp16 outputs of row m in
// columns [128 j, 128 j + 128) -- the row statistic of the next norm-folded projection without a
// pass over the hidden state (fls_rstd_from_ss)
// rstd[r] = rsqrt(sum_j ss[r * ss_ld + j] / H + eps) for j < nparts, summed in a fixed order
int fls_row_stat(const void* x, int ldx, int rows, int H, float eps, float* rstd, fls_stream_t s);  // row_ss + rstd_from_ss, fused
int fls_row_ss(const void* x, int ldx, int rows, int H, float* ss, int ss_ld, fls_stream_t s);  // residual-epilogue partials of x
int fls_rstd_from_ss(const float* ss, int ss_ld, int nparts, int rows, int H, float eps, float* rstd,
                     fls_stream_t s);
// out[r] = first index of the maximum of row r of non-negative fp16 values (greedy decoding)
int fls_argmax_rows(const void* x, int ld, int rows, int V, int* out, fls_stream_t s);
// rstd[r] = rsqrt(mean(x[row]^2) + eps) in fp32, row = row_idx ? row_idx[r] : r (fused RMSNorm:
// the statistic of the rows a norm-folded projection reads raw)
int fls_row_rstd(const void* x, int ldx, const int* row_idx, int rows, int H, float eps, float* rstd,
                 fls_stream_t s);
// W[n, k] = fp16(W[n, k] * gamma[k]) in place for n < N, k < K (the RMSNorm weight folded into
// the projection that consumes the normed rows)
int fls_fold_norm(void* w, int ldw, int N, int K, const void* gamma, fls_stream_t s);
// y[dst_idx[r]] = x[src_idx[r]] for r < rows (fp16 rows of H elements; a null index = identity)
// device-to-device copy: mode 0 HIP runtime (blit kernel), 1 SDMA engines (no CU), 2 `blocks` workgroups
int fls_copy_d2d(void* dst, const void* src, uint64_t bytes, int mode, int blocks, fls_stream_t s);
int fls_copy_rows(const void* x, int ldx, const int* src_idx, void* y, int ldy, const int* dst_idx, int rows, int H,
                  fls_stream_t s);
int fls_gemm_set_splitk(int on);
int fls_gemm_set_row_chunk(int rows);   // rows per main-path GEMM launch (default 16384; 0 = unlimited)
// mixture-of-experts FFN (csrc/kernels/moe.hip): routing, stable expert sort, grouped v10 GEMM
// (every expert of a layer in one launch, optional row gather), fp16-ordered weighted combine
int fls_moe_route(const void* logits, int ldl, int T, int E, int k, int norm, int round16, int* ids, float* w,
                  fls_stream_t s);
int fls_moe_router_route(const void* h, int ldh, const void* wr, int ldw, int T, int H, int E, int k, int norm,
                         int round16, int* ids, float* w, fls_stream_t s);   // router logits fused (E <= 64)
int fls_moe_plan_scratch(int n, int E);   // ints of the bhist scratch fls_moe_plan needs
int fls_moe_plan(const int* ids, int n, int k, int E, int* offs, int* tiles, int* rows, int* dest, int* bhist,
                 fls_stream_t s);
int fls_moe_gemm(const void* A, const void* W, void* C, int M_bound, int N, int K, int lda, int ldw, int ldc, int epi,
                 const int* tiles, const int* offs, const int* rows, int n_groups, long long wstride, int a_rows,
                 fls_stream_t s);
int fls_moe_combine(const void* y, int ldy, const int* ids, const int* dest, const float* w, void* x, int ldx, int T,
                    int k, int H, const void* sh, int ldsh, fls_stream_t s);   // sh: optional shared-expert term
int fls_gemm_set_order(int order);   // tile order: 0 by shape, 8 M-grouped, -4/-8 N-grouped
int fls_gemm_set_mid_bn(int bn);     // mid-M block columns: 0 auto, 64 / 128 forced
int fls_gemm_set_mid_waves(int waves);  // 128-column mid-M blocks: 0 auto, 4 / 8 waves forced
int fls_gemm_set_mid_rows(int rows);  // 8-wave mid-M blocks: rows, 0 auto, 64 / 128 forced
int fls_gemm_set_mid(int on);   // 64x128-tile kernel for small / medium M (default on)
// shared-prefix / varlen flash attention over packed work items (int32 x8:
// q_start q_len q_off r0_start r0_len r0_causal r1_start r1_len).
// kv0 (optional, [P, 2*n_kv*hd] K then V, row stride ld_kv0): range 0 of every work item indexes it.
// seg_lo (optional, [T] int32): first packed row of the suffix holding each row; range-1 key j is
// visible to query row i iff seg_lo[i] <= j <= i, so an item may hold several suffixes of a prompt
// (null: one suffix per item).  q_block: rows per work item (64 or 128).
// work2 (optional, int32 x2 per item: r2_start r2_len): range 2 = kv0 rows [r2_start, +r2_len) walked
// between range 0 and range 1, of which query row i sees kv0 rows [r2win[2i], r2win[2i+1]) (its
// suffix's cached K/V rows; needs kv0 and r2win).
int fls_attention_set_hpb(int hpb);
int fls_attention_set_split(int ns);
int fls_attention_set_persistent(int on);   // persistent full-pass kernel (default on; tests / A-B)
// ws / ws_bytes / n_rows (rows of qkv and out): fp32 scratch of the split-KV range-2 kernel (null: no split)
int fls_attention(const void* qkv, void* out, const int* work, int n_items, int n_q_heads,
                  int n_kv_heads, int head_dim, int ld_qkv, int ld_out, float scale, const void* kv0,
                  int ld_kv0, const int* seg_lo, int q_block, const int* work2, const int* r2win,
                  void* ws, unsigned long long ws_bytes, int n_rows, fls_stream_t s);
int fls_headnorm_rope(void* x, int ldx, int rows, int n_q, int n_k, const void* qn, const void* kn, const int* pos,
                      const float* cos_t, const float* sin_t, int hd, float eps, fls_stream_t s);
int fls_rmsnorm(const void* x, const void* w, void* y, const int* row_idx, int rows, int H,
                int ldx, int ldy, float eps, fls_stream_t s);
int fls_embed(const int* ids, const void* table, void* out, int T, int H, int V, float scale, fls_stream_t s);
int fls_softmax_rows(const void* logits, void* probs, int rows, int V, float inv_scale, fls_stream_t s);
// dst = fp16(src): src_dtype 1 = bf16 (in place allowed), 2 = fp32 (no overlap)
int fls_cast_f16(void* dst, const void* src, int src_dtype, uint64_t n, fls_stream_t s);
// C[M,N] = X[M,K] W[N,K]^T for M <= 16 (skinny LM head); K % 32 == 0
int fls_gemv_skinny(const void* x, const void* w, void* c, int M, int N, int K, int ldx, int ldw, int ldc,
                    fls_stream_t s);
int fls_fill_random(void* dst, uint64_t n_elems, uint64_t seed, float mean, float std,
                    fls_stream_t s);

#ifdef __cplusplus
}
#endif
