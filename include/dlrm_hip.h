/*
 * dlrm_hip.h — C-ABI of the MI355X-native (gfx950) DLRM training hot path.
 *
 * This is the drop-in boundary between the Python host layer (a mirror of the
 * reference's DLRM_Net / TableBatchedEmbeddingBags / ext_dist surface) and the
 * hand-written CDNA4 HIP kernels in dlrm-yx_amd/csrc.  Every entry point:
 *   - takes plain device pointers, sizes and a hipStream_t (no torch types);
 *   - enqueues asynchronously on the caller's stream and never synchronises,
 *     allocates or frees device memory (workspaces come from the caller, sized
 *     by the *_workspace_size() queries) — so every call is hipGraph-capturable;
 *   - returns an int status (DLRM_OK == 0) and never exit()s; the message for
 *     the last failure on the calling thread is in dlrm_last_error();
 *   - is reentrant: no mutable global state.
 *
 * Reference interfaces replaced (file:line in YuxinxinChen/dlrm-yx):
 *   dlrm_tbe_forward          <- torch.ops.batched_forward.forward
 *                                (yx_modfs/batched_forward.cpp:4-13,
 *                                 yx_modfs/table_batched_embeddings_cuda_yx.cu:317-389)
 *                                and nn.EmbeddingBag(mode="sum") forward as called by
 *                                DLRM_Net.apply_emb (dlrm_s_pytorch.py:526-587),
 *                                TableBatchedEmbeddingBags.__call__ (dlrm_s_pytorch.py:321-334,589-591)
 *   dlrm_tbe_backward_sgd     <- EmbeddingBag sparse backward + torch.optim.SGD sparse
 *                                add_ (dlrm_s_pytorch.py:1923-1934), i.e. the exact-SGD
 *                                TBE backward of create_emb_batched (dlrm_s_pytorch.py:321-334)
 *   dlrm_tbe_backward_rowwise_adagrad
 *                             <- RWSAdagrad.step sparse branch (optim/rwsadagrad.py:92-115)
 *   dlrm_qr_split_indices / dlrm_qr_combine_* <- QREmbeddingBag.forward
 *                                (tricks/qr_embedding_bag.py:156-174)
 *   dlrm_interact_dot_*       <- DLRM_Net.interact_features, "dot" branch
 *                                (dlrm_s_pytorch.py:627-659)
 *   dlrm_interact_cat_*       <- DLRM_Net.interact_features, "cat" branch
 *                                (dlrm_s_pytorch.py:660-665)
 *   dlrm_gemm_f32             <- nn.Linear (+ReLU) forward/backward inside
 *                                DLRM_Net.create_mlp/apply_mlp (dlrm_s_pytorch.py:227-265,518-524)
 *   dlrm_colsum_f32           <- Linear bias gradient (sum over the batch)
 *   dlrm_head_forward_backward<- last Linear + Sigmoid + loss_fn_wrap (mse/bce)
 *                                (dlrm_s_pytorch.py:170-178,504-516,1907)
 *   dlrm_sgd_update / dlrm_adagrad_update
 *                             <- torch.optim.SGD.step dense branch / RWSAdagrad dense
 *                                branch (optim/rwsadagrad.py:117-120)
 *   dlrm_uniform_fill         <- np.random.uniform table init (dlrm_s_pytorch.py:304-308),
 *                                device-side for tables too large for host init
 *   dlrm_csr_from_tables      <- table-batched CSR flatten (dlrm_data_pytorch.py:748-753,834-843)
 *   dlrm_criteo_decode        <- CriteoBinDataset.__getitem__ + _transform_features
 *                                (data_loader_terabyte.py:83-114,237-252)
 */
#ifndef DLRM_HIP_H_
#define DLRM_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* hipStream_t is an opaque pointer; declared here so the header needs no HIP headers. */
typedef struct ihipStream_t* dlrm_stream_t;

enum dlrm_status {
  DLRM_OK = 0,
  DLRM_ERR_INVALID_ARG = 1, /* null pointer / bad enum / negative size          */
  DLRM_ERR_SHAPE = 2,       /* inconsistent shapes or alignment                 */
  DLRM_ERR_UNSUPPORTED = 3, /* shape the kernels do not handle                  */
  DLRM_ERR_WORKSPACE = 4,   /* workspace smaller than *_workspace_size()        */
  DLRM_ERR_HIP = 5          /* a HIP launch/runtime error                       */
};

/* GEMM epilogues (C[m][n] <- f(alpha * acc[m][n], ...)). */
enum dlrm_epilogue {
  DLRM_EPI_STORE = 0,     /* C = alpha*acc                                      */
  DLRM_EPI_BIAS = 1,      /* C = alpha*acc + bias[n]                            */
  DLRM_EPI_BIAS_RELU = 2, /* C = max(alpha*acc + bias[n], 0)      (Linear+ReLU) */
  DLRM_EPI_DRELU = 3,     /* C = alpha*acc * (aux[m][n] > 0)      (ReLU bwd)    */
  DLRM_EPI_SGD = 4,       /* C = C - alpha*acc                    (fused SGD)   */
  DLRM_EPI_ACCUM = 5,     /* C = C + alpha*acc                                  */
  DLRM_EPI_RELU = 6       /* C = max(alpha*acc, 0)   (Linear+ReLU, bias folded) */
};

enum dlrm_loss { DLRM_LOSS_MSE = 0, DLRM_LOSS_BCE = 1 };

/* Bits a TBE launch ORs into its device error_flag (int32; the caller zeroes it and
 * reads it when convenient — the launches never synchronise). */
enum dlrm_tbe_error {
  DLRM_TBE_ERR_INDEX = 1,    /* an index outside [0, rows of its table): the lookup
                                contributed nothing / received no update             */
  DLRM_TBE_ERR_TABLE_CAP = 2 /* backward: a table had more lookups than the caller's
                                max_lookups_per_table; that table was not updated     */
};

enum dlrm_qr_op { DLRM_QR_MULT = 0, DLRM_QR_ADD = 1, DLRM_QR_CONCAT = 2 };

/* ---------------------------------------------------------------- library -- */
/* 2: the TBE backward entry points take an error_flag (round 2).
 * 3: dlrm_qr_expand_csr takes phys_capacity + error_flag; a PARTIAL split count must be
 *    normalized (dlrm_gemm_f32_splits) (round 3).
 * 4: dlrm_gemm_problem carries split-bf16 planes; dlrm_split_planes; the TBE backward's
 *    rows per call must be < 2^32 - 1 (round 3).
 * 5: the split-bf16 planes and dlrm_split_planes are gone again (measured slower than the
 *    exact-f32 MFMA path in the step, profiles/r03_planes_*.txt): dlrm_gemm_problem ends
 *    at `partial`; dlrm_tbe_forward_presort's out = NULL (sort-only) mode is used by the
 *    engine (round 4).
 * 6: dlrm_tbe_backward_defer + dlrm_gemm_f32_group_role: the embedding backward's update
 *    passes (and dlrm_tbe_sort_defer: the per-table sort; dlrm_head_step_defer: the head's
 *    finalize pass) as extra workgroups of grouped GEMM launches (dlrm_launch_role); dlrm_mlp_chain gains parts /
 *    split_layer / tickets (several workgroups per 16-row block) (round 4).
 * 7: dlrm_tbe_sort_defer and role phase 3 removed (the sort as a GEMM-launch role measured
 *    slower than the sort in the lookup launch everywhere, profiles/r04_sort_role_ab.txt)
 *    (round 5).
 * 8: dlrm_mlp_chain_backward removed (the bottom MLP's data gradients as one row-block
 *    launch lost to the grouped GEMM schedules at every batch size,
 *    profiles/r04_bot_sched_ab.txt) (round 5).
 * 9: dlrm_adagrad_update_scaled (the W-rank dense Adagrad step with the 1/W folded in)
 *    (round 6).
 * 10: dlrm_tbe_backward_sort + presorted = DLRM_PRESORTED_ANY (the backward's sort run
 *    early, e.g. on a second stream) (round 6). */
#define DLRM_ABI_VERSION 10 /* the one source of truth: abi.cpp returns it, dlrm_hip/_lib.py
                             pins it (tests/test_cpu_host.py checks all of them agree) */
int dlrm_abi_version(void);
const char* dlrm_last_error(void);

/* Plan overrides for autotuning sweeps and coverage tests (ABI v5; the library reads no
 * environment).  THREAD-LOCAL: they apply to the calls the calling host thread makes;
 * value 0 restores the planner's choice.  Results stay exact under any override (the
 * tests compare every path with the reference), only speed changes.
 *   DLRM_TUNE_GEMM_TILE  : BM * 1000 + BN of the pipelined GEMM's workgroup tile (64064,
 *                          128064, 64128, 32064, 64032, 32032); the measured plan table is skipped
 *   DLRM_TUNE_GEMM_SPLIT : K splits of every FULL problem (with DLRM_TUNE_GEMM_TILE)
 *   DLRM_TUNE_TBE_BLOCK  : sorted lookups per TBE-backward block (16 or 64)
 *   DLRM_TUNE_TBE_SORT   : 1 = the device-wide radix sort even where the tiled per-table
 *                          sort applies; 2 = the tiled passes' digit scan as the chunked
 *                          (csum / scan) launches instead of the wide scan (ABI v6)
 *   DLRM_TUNE_TBE_LEAN   : 1 = the non-deferred backward's update passes as the
 *                          16-rows-in-flight kernels even where the lean ones apply (ABI v6)
 *   DLRM_TUNE_INTERACT_BWD : the dot-interaction backward's kernel: 3 = one wave per sample
 *                          (v3), 4 = one wave per sample x 32-column block (v4), 5 = one
 *                          workgroup per sample, a wave per 32-column block (v5, D >= 64);
 *                          default v4 for D <= 32; above, v5 for batches <= 1024, else v3
 *                          (ABI v6; v5 in v7)
 *   DLRM_TUNE_INTERACT_FWD : the dot-interaction forward's kernel: 4 = one wave per sample
 *                          (v4), 5 = one workgroup per sample (v5, D >= 64; default there
 *                          for batches <= 1024)
 *                          (ABI v7) */
enum dlrm_tune_key {
  DLRM_TUNE_GEMM_TILE = 1,
  DLRM_TUNE_GEMM_SPLIT = 2,
  DLRM_TUNE_TBE_BLOCK = 3,
  DLRM_TUNE_TBE_SORT = 4,
  DLRM_TUNE_TBE_LEAN = 5,
  DLRM_TUNE_INTERACT_BWD = 6,
  DLRM_TUNE_INTERACT_FWD = 7
};
int dlrm_set_tuning(int32_t key, int64_t value);
int64_t dlrm_get_tuning(int32_t key);

/* ------------------------------------------------ table-batched embedding -- */
/*
 * Pooled-sum lookup for T tables stored row-concatenated in one [total_rows][D]
 * fp32 buffer.  Table t owns rows [row_base[t], row_base[t+1]) (row_base: device
 * int64 [T+1]).  Bags are the CSR of the reference's batched layout: bag
 * (t, b) = t*B + b covers lookups [offsets[bag], offsets[bag+1]), offsets has
 * T*B+1 entries (device, int32 or int64 by offset_bits), indices are table-local
 * rows (device, int32 or int64 by index_bits).
 *   out[b*out_batch_stride + t*D + d] = sum_l w_l * W[row_base[t] + indices[l]][d]
 * (w_l = per_sample_weights[l], or 1 when per_sample_weights == NULL), summed in
 * lookup order in fp32.  An out-of-range index contributes nothing and ORs
 * DLRM_TBE_ERR_INDEX into *error_flag (error_flag may be NULL).
 */
int dlrm_tbe_forward(const float* weights, int64_t D, const int64_t* row_base, int32_t T,
                     int32_t B, const void* indices, int32_t index_bits, const void* offsets,
                     int32_t offset_bits, const float* per_sample_weights, float* out,
                     int64_t out_batch_stride, int32_t* error_flag, dlrm_stream_t stream);

/*
 * A Linear+ReLU stack with the bias folded into the weights (the trainer's layout of the
 * bottom MLP, DLRM_Net.create_mlp / apply_mlp, dlrm_s_pytorch.py:227-265, 518-524):
 *   Y_l[r][c] = relu(sum_{k < in_width[l]} In_l[r][k] * W_l[c][k]),  c < out_width[l]
 * with In_0 = X (which carries its own bias column) and, for l > 0, In_l = Y_{l-1} with
 * column out_width[l-1] = 1 and the remaining padding 0; in_width[l] =
 * pad4(out_width[l-1] + 1).  Only columns < out_width[l] of Y_l are written.  Supported
 * (dlrm_mlp_chain_supported): 1..4 layers, out_width <= 512, in_width rounded up to 16
 * <= 528, X and W 16-byte aligned with row strides % 4 == 0.
 * parts (ABI v6; 0 or 1 = off): 2 or 4 workgroups share each 16-row block.  Layer
 * split_layer's 16-column tiles are dealt out between them (each needs >= 1 tile), the
 * layers before it are computed by every part (only part 0 writes their Y), and when
 * split_layer is not the last layer the part that finishes its columns last - an
 * agent-scope ticket in tickets[block], int32 [ceil(rows / 16)], zero before the first call
 * and left zero by every call - reads the other parts' columns of Y_split (published
 * write-through) and runs the remaining layers.  Same result as parts = 1, bit for bit:
 * every output element is the same dot product in the same order.  Tickets are per chain:
 * two launches in flight at once must not share them.
 */
#define DLRM_MLP_MAX_LAYERS 4
typedef struct dlrm_mlp_chain {
  int32_t layers;
  int64_t rows;
  const float* X;
  int64_t ldx;
  int64_t in_width[DLRM_MLP_MAX_LAYERS];
  int64_t out_width[DLRM_MLP_MAX_LAYERS];
  const float* W[DLRM_MLP_MAX_LAYERS];
  int64_t ldw[DLRM_MLP_MAX_LAYERS];
  float* Y[DLRM_MLP_MAX_LAYERS];
  int64_t ldy[DLRM_MLP_MAX_LAYERS];
  int32_t parts;       /* ABI v6 */
  int32_t split_layer; /* ABI v6 */
  int32_t* tickets;    /* ABI v6 */
} dlrm_mlp_chain;

/* 1 when dlrm_mlp_chain_forward / the fused forward can take this chain, else 0. */
int dlrm_mlp_chain_supported(const dlrm_mlp_chain* chain);

/* The chain on its own: 16 rows per workgroup, every layer in one launch. */
int dlrm_mlp_chain_forward(const dlrm_mlp_chain* chain, dlrm_stream_t stream);

/*
 * dlrm_tbe_forward + the per-table sort of the backward (which depends only on the
 * indices) in ONE launch: the sort's latency-bound workgroups run beside the gather.
 * The sort lands in `workspace` (a dlrm_tbe_backward_* workspace); call the backward of
 * the same batch with presorted = 1.  When the per-table sort does not apply (64-bit row
 * ids, max_lookups_per_table 0 or > 4096) this is dlrm_tbe_forward and the backward
 * sorts as usual.
 * bottom != NULL: the bottom MLP forward (an independent input of the same step) runs as
 * a third role of the same launch (dlrm_mlp_chain semantics; it must be supported); when
 * the presort does not apply it still shares the lookup launch (round 6; D <= 512, out != NULL;
 * otherwise its own launch after the lookup).
 * out == NULL (round 3): no lookup role - its consumer gathers the rows itself
 * (dlrm_interact_dot_forward_gather); needs the per-table sort to apply (else UNSUPPORTED).
 */
int dlrm_tbe_forward_presort(const float* weights, int64_t D, const int64_t* row_base, int32_t T,
                             int32_t B, const void* indices, int32_t index_bits,
                             const void* offsets, int32_t offset_bits,
                             const float* per_sample_weights, float* out,
                             int64_t out_batch_stride, int64_t num_lookups, int64_t total_rows,
                             int64_t max_lookups_per_table, void* workspace,
                             size_t workspace_bytes, int32_t* error_flag,
                             const dlrm_mlp_chain* bottom, dlrm_stream_t stream);

/*
 * Reduced-precision rows.  Row layouts, fixed row_bytes per buffer:
 *   DLRM_ROWS_F16 : D fp16 (the fbgemm TBE's FP16 weights, dlrm_s_pytorch.py:337-366)
 *   DLRM_ROWS_Q8  : D uint8, fp32 scale, fp32 bias (torch.ops.quantized
 *                   .embedding_bag_byte_prepack, dlrm_s_pytorch.py:609-625)
 *   DLRM_ROWS_Q4  : ceil(D/2) bytes (element 2i = low nibble of byte i), fp16 scale, fp16
 *                   bias (embedding_bag_4bit_prepack)
 * value = q * scale + bias.
 */
enum dlrm_rows_format {
  DLRM_ROWS_F32 = 0,
  DLRM_ROWS_F16 = 1,
  DLRM_ROWS_Q8 = 2,
  DLRM_ROWS_Q4 = 3
};

/* Minimum row size in bytes of a format at dimension D (-1 for an unknown format). */
int64_t dlrm_tbe_row_bytes(int32_t format, int64_t D);

/*
 * dlrm_tbe_forward over F16 / Q8 / Q4 rows (embedding_bag_{byte,4bit}_rowwise_offsets
 * semantics, dlrm_s_pytorch.py:554-567, table-batched like dlrm_tbe_forward): each bag
 * sums fma(w*scale, q, acc + w*bias) in fp32.  weights: [total_rows][row_bytes] bytes;
 * D % 4 == 0, D <= 512; rows 8- (F16), 4- (Q8) or 2-byte (Q4) aligned.
 */
int dlrm_tbe_forward_rows(const void* weights, int32_t format, int64_t row_bytes, int64_t D,
                          const int64_t* row_base, int32_t T, int32_t B, const void* indices,
                          int32_t index_bits, const void* offsets, int32_t offset_bits,
                          const float* per_sample_weights, float* out, int64_t out_batch_stride,
                          int32_t* error_flag, dlrm_stream_t stream);

/*
 * Gradient of the per-sample weights of a weighted lookup (learned weighted pooling,
 * dlrm_s_pytorch.py:475-478, 544-545): grad_per_sample_weights[l] =
 * sum_d grad_out[b*grad_batch_stride + t*D + d] * W[row_base[t] + indices[l]][d] for the
 * bag (t, b) holding lookup l (0 for lookups outside every bag or out of range).
 */
int dlrm_tbe_psw_grad(const float* weights, int64_t D, const int64_t* row_base, int32_t T,
                      int32_t B, const void* indices, int32_t index_bits, const void* offsets,
                      int32_t offset_bits, int64_t num_lookups, const float* grad_out,
                      int64_t grad_batch_stride, float* grad_per_sample_weights,
                      dlrm_stream_t stream);

/* Workspace for the deterministic (sorted, segment-reduced) backward. */
size_t dlrm_tbe_backward_workspace_size(int64_t num_lookups, int64_t total_rows, int64_t D);

/*
 * ABI v10: the sort phase of the backward alone (whichever sort the backward would run for
 * the same D, tables, indices, offsets, bound, workspace and per_sample_weights nullness:
 * per-table, tiled per-table, or device-wide), into `workspace`.  It depends only on the
 * indices, so a caller can run it early - e.g. on a second stream beside the forward - and
 * then call the backward of the same batch with presorted = DLRM_PRESORTED_ANY.
 */
#define DLRM_PRESORTED_ANY 2
int dlrm_tbe_backward_sort(int64_t D, const int64_t* row_base, int32_t T, int32_t B,
                           const void* indices, int32_t index_bits, const void* offsets,
                           int32_t offset_bits, int64_t num_lookups, int64_t total_rows,
                           const float* per_sample_weights, int64_t max_lookups_per_table,
                           void* workspace, size_t workspace_bytes, int32_t* error_flag,
                           dlrm_stream_t stream);

/*
 * Exact-SGD backward fused with the update: for every lookup l of bag (t,b),
 *   W[row_base[t]+indices[l]] -= lr * w_l * grad_out[b*grad_batch_stride + t*D + :]
 * Duplicate rows are combined deterministically: lookups are sorted by (global row,
 * position), the gradient of each unique row is summed in sorted order (long runs in
 * fixed 16-lookup blocks whose partials are added in block order), and the row is
 * read once and written once.  num_lookups = length of indices.
 * max_lookups_per_table: an upper bound on the lookups of any single table in this
 * call (B*L for fixed bag size L), or 0 if unknown.  With 32-bit row ids and a bound
 * <= 4096 each table is sorted in LDS by one workgroup; otherwise a device-wide radix
 * sort is used.  A bound smaller than the real maximum is a contract violation: the
 * offending table is skipped and DLRM_TBE_ERR_TABLE_CAP is set in *error_flag.
 * Out-of-range indices are skipped and set DLRM_TBE_ERR_INDEX (the reference's
 * EmbeddingBag raises IndexError there).  error_flag may be NULL.
 * presorted != 0: the per-table sort of THIS batch (same indices, offsets, workspace)
 * already ran inside dlrm_tbe_forward_presort and is skipped here (ignored when the
 * per-table sort does not apply: 32-bit row ids, bound <= 4096).
 * presorted == DLRM_PRESORTED_ANY (ABI v10): dlrm_tbe_backward_sort already ran for THIS
 * batch with the same arguments; whichever sort applies is skipped.
 * (The same applies to the two functions below.)
 */
int dlrm_tbe_backward_sgd(float* weights, int64_t D, const int64_t* row_base, int32_t T,
                          int32_t B, const void* indices, int32_t index_bits,
                          const void* offsets, int32_t offset_bits, int64_t num_lookups,
                          int64_t total_rows, const float* per_sample_weights,
                          const float* grad_out, int64_t grad_batch_stride, float lr,
                          int64_t max_lookups_per_table, void* workspace,
                          size_t workspace_bytes, int32_t* error_flag, int32_t presorted,
                          dlrm_stream_t stream);

/*
 * dlrm_tbe_backward_sgd on fp16 weights (DLRM_ROWS_F16 tables: the fbgemm TBE's FP16
 * weights with EXACT_SGD, dlrm_s_pytorch.py:337-366): the gradient of each unique row is
 * summed in fp32 in the same fixed order, w = float(w_fp16) - lr * g is rounded to nearest
 * even on the store (fbgemm's optional stochastic rounding is not reproduced).
 */
int dlrm_tbe_backward_sgd_f16(void* weights, int64_t D, const int64_t* row_base, int32_t T,
                              int32_t B, const void* indices, int32_t index_bits,
                              const void* offsets, int32_t offset_bits, int64_t num_lookups,
                              int64_t total_rows, const float* per_sample_weights,
                              const float* grad_out, int64_t grad_batch_stride, float lr,
                              int64_t max_lookups_per_table, void* workspace,
                              size_t workspace_bytes, int32_t* error_flag, int32_t presorted,
                              dlrm_stream_t stream);

/*
 * Row-wise sparse Adagrad (RWSAdagrad, optim/rwsadagrad.py:92-115) fused into the
 * backward: per unique row r with coalesced gradient g_r (sum over its lookups),
 *   momentum[r] += mean_d(g_r[d]^2);  W[r] -= lr * g_r / (sqrt(momentum[r]) + eps)
 * momentum: device fp32 [total_rows].
 */
int dlrm_tbe_backward_rowwise_adagrad(float* weights, float* momentum, int64_t D,
                                      const int64_t* row_base, int32_t T, int32_t B,
                                      const void* indices, int32_t index_bits,
                                      const void* offsets, int32_t offset_bits,
                                      int64_t num_lookups, int64_t total_rows,
                                      const float* per_sample_weights, const float* grad_out,
                                      int64_t grad_batch_stride, float lr, float eps,
                                      int64_t max_lookups_per_table, void* workspace,
                                      size_t workspace_bytes, int32_t* error_flag,
                                      int32_t presorted, dlrm_stream_t stream);

/*
 * Dense (non-fused) embedding-bag gradient scatter: grad_weights[row] += w_l * g
 * for every lookup, deterministic (same sort), into a zero-initialised (or
 * accumulating) [total_rows][D] buffer.  Used when the caller owns the optimizer.
 */
int dlrm_tbe_backward_dense(float* grad_weights, int64_t D, const int64_t* row_base,
                            int32_t T, int32_t B, const void* indices, int32_t index_bits,
                            const void* offsets, int32_t offset_bits, int64_t num_lookups,
                            int64_t total_rows, const float* per_sample_weights,
                            const float* grad_out, int64_t grad_batch_stride,
                            int64_t max_lookups_per_table, void* workspace,
                            size_t workspace_bytes, int32_t* error_flag, int32_t presorted,
                            dlrm_stream_t stream);

/*
 * Deferred update (ABI v6): dlrm_tbe_backward_sgd (mode 0) or
 * dlrm_tbe_backward_rowwise_adagrad (mode 1, momentum required) with the same arguments,
 * except that the two update passes - the block pass over the sorted lookups and the
 * combine pass over runs that cross blocks - are not launched: *role receives them, to
 * run as extra workgroups of two later launches, phase 1 then phase 2, via
 * dlrm_gemm_f32_group_role (typically the bottom-MLP backward's GEMM launches, which touch
 * none of the TBE's buffers: the HBM-bound update overlaps the MFMA-bound GEMMs with no
 * cross-stream dependency).  Everything before the passes (the sort, unless presorted)
 * is launched here.  The result is bitwise the non-deferred call's.  role->blocks == 0
 * after the call (not covered: D != 4*LPB for LPB in 4..32, unaligned rows, per-sample
 * weights, B * grad_batch_stride >= 2^31, N == 0): the update ran in full here and the
 * role passes are no-ops.  Until both phases have run, the workspace,
 * weights, momentum and grad_out must stay as they are.
 */
typedef struct dlrm_launch_role {
  uint64_t opaque[32];
} dlrm_launch_role;
int dlrm_tbe_backward_defer(int32_t mode, float* weights, float* momentum, int64_t D,
                            const int64_t* row_base, int32_t T, int32_t B,
                            const void* indices, int32_t index_bits, const void* offsets,
                            int32_t offset_bits, int64_t num_lookups, int64_t total_rows,
                            const float* per_sample_weights, const float* grad_out,
                            int64_t grad_batch_stride, float lr, float eps,
                            int64_t max_lookups_per_table, void* workspace,
                            size_t workspace_bytes, int32_t* error_flag, int32_t presorted,
                            dlrm_launch_role* role, dlrm_stream_t stream);
/* Workgroups a deferred pass adds to the launch that carries it (0: nothing deferred). */
int32_t dlrm_role_blocks(const dlrm_launch_role* role);
/*
 * Sparse-gradient values of an EmbeddingBag(sparse=True) backward
 * (torch _embedding_bag_sparse_backward as reached from dlrm_s_pytorch.py:1929):
 *   values[l][:] = w_l * grad_out[b*grad_batch_stride + t*D + :] for lookup l of bag (t,b)
 * values: [num_lookups][D]; lookups outside every bag get zeros.
 */
int dlrm_tbe_expand_grad(int64_t D, int32_t T, int32_t B, const void* offsets,
                         int32_t offset_bits, int64_t num_lookups,
                         const float* per_sample_weights, const float* grad_out,
                         int64_t grad_batch_stride, float* values, dlrm_stream_t stream);

/* -------------------------------------------------- QR embeddings (C4) ---- */
/* q[l] = trunc((float)idx[l] / (float)collisions), r[l] = idx[l] mod collisions
 * (tricks/qr_embedding_bag.py:157-158 semantics, float division included). */
int dlrm_qr_split_indices(const void* indices, int32_t index_bits, int64_t n,
                          int64_t collisions, int64_t* q_out, int64_t* r_out,
                          dlrm_stream_t stream);
/* out = op(eq, er) elementwise over n_rows rows of D (concat: out row = [eq|er]). */
int dlrm_qr_combine_forward(int32_t op, int64_t n_rows, int64_t D, const float* eq,
                            const float* er, float* out, dlrm_stream_t stream);
int dlrm_qr_combine_backward(int32_t op, int64_t n_rows, int64_t D, const float* eq,
                             const float* er, const float* grad_out, float* grad_eq,
                             float* grad_er, dlrm_stream_t stream);

/* Table-batched QR for the fused engine (create_emb's QR branch, dlrm_s_pytorch.py:282-290,
 * on the batched CSR): physical table p takes the bags of logical table src[p] with the
 * logical indices (kind 0), the quotients trunc((float)idx / coll[p]) (kind 1) or the
 * remainders idx mod coll[p] (kind 2) -> int32 phys_indices / phys_offsets[T_phys*B+1].
 * src / kind / coll are DEVICE int32 arrays of T_phys entries.  phys_indices holds
 * phys_capacity entries: lookups past it are dropped, the offsets are clamped to it (the
 * bags stay well formed) and DLRM_TBE_ERR_TABLE_CAP is set in *error_flag (may be NULL). */
int dlrm_qr_expand_csr(int32_t T_phys, int32_t B, const void* indices, int32_t index_bits,
                       const void* offsets, int32_t offset_bits, const int32_t* src,
                       const int32_t* kind, const int32_t* coll,
                       int64_t max_lookups_per_table, int32_t* phys_indices,
                       int32_t* phys_offsets, int64_t phys_capacity, int32_t* error_flag,
                       dlrm_stream_t stream);
/* E[b][t] = op(P[b][pq[t]], P[b][pr[t]]) (QREmbeddingBag.forward's combine,
 * tricks/qr_embedding_bag.py:166-172; op mult or add) for pr[t] >= 0, else P[b][pq[t]];
 * P: pooled physical tables [B][.][D] (row stride p_batch_stride), E: [B][T][D].
 * pq / pr: DEVICE int32 [T].  D and the strides are multiples of 4. */
int dlrm_qr_pool_combine_forward(int32_t op, int32_t T, int64_t B, int64_t D, const int32_t* pq,
                                 const int32_t* pr, const float* P, int64_t p_batch_stride,
                                 float* E, int64_t e_batch_stride, dlrm_stream_t stream);
/* dP[b][pq[t]] = dE * P[b][pr[t]], dP[b][pr[t]] = dE * P[b][pq[t]] (mult; add: dE to both);
 * dP[b][pq[t]] = dE for tables without a remainder. */
int dlrm_qr_pool_combine_backward(int32_t op, int32_t T, int64_t B, int64_t D,
                                  const int32_t* pq, const int32_t* pr, const float* P,
                                  int64_t p_batch_stride, const float* dE,
                                  int64_t e_batch_stride, float* dP, int64_t dp_batch_stride,
                                  dlrm_stream_t stream);

/* ------------------------------------------------------------ interaction -- */
/*
 * Feature f of sample b lives at feat_ptrs[f] + b*feat_bstrides[f] (D floats);
 * feature 0 is the bottom-MLP output.  feat_ptrs / feat_bstrides are HOST arrays
 * of F entries (copied into kernel arguments; F <= 64).
 * Dot: out[b][0:D] = feature0, out[b][D + p] = <T_i, T_j> for the p-th pair of the
 * row-major lower triangle (i > j, or i >= j when self_interaction), as
 * torch.tril_indices(F, F, -1 or 0).
 */
int dlrm_interact_dot_forward(int32_t B, int32_t F, int32_t D, const float* const* feat_ptrs,
                              const int64_t* feat_bstrides, int32_t self_interaction,
                              float* out, int64_t ld_out, dlrm_stream_t stream);
/* Writes (overwrites) grad of every feature: grad_ptrs[f] + b*grad_bstrides[f].
 * relu_x != 0 also applies ReLU'(x) to feature 0's gradient (x = the bottom MLP's ReLU
 * output: the backward of that ReLU, fused). */
int dlrm_interact_dot_backward(int32_t B, int32_t F, int32_t D,
                               const float* const* feat_ptrs, const int64_t* feat_bstrides,
                               int32_t self_interaction, const float* grad_out,
                               int64_t ld_gout, float* const* grad_ptrs,
                               const int64_t* grad_bstrides, int32_t relu_x,
                               dlrm_stream_t stream);

/*
 * The one-hot lookup fused into the dot interaction (one GPU, L = 1: apply_emb with one
 * index per bag, dlrm_s_pytorch.py:526-587, then interact_features :627-659): feature 0 is
 * x (x_bstride floats per sample), feature f >= 1 of sample b is row
 * row_base[f-1] + indices[(f-1) * B + b] of `weights` (table-major CSR indices; row_base
 * DEVICE int64 [F], its last entry the total row count).  An index outside its table
 * reads as a zero row (the TBE drops it from its bag) and sets DLRM_TBE_ERR_INDEX in
 * *error_flag (may be NULL).  Output as dlrm_interact_dot_forward; the [B, T, D] pooled
 * embeddings are never written.  D in {16, 32, 64, 128}, 2 <= F <= 32, x / weights 16-B
 * aligned (else UNSUPPORTED / INVALID_ARG).
 */
int dlrm_interact_dot_forward_gather(int32_t B, int32_t F, int32_t D, const float* x,
                                     int64_t x_bstride, const float* weights,
                                     const int64_t* row_base, const int32_t* indices,
                                     int32_t self_interaction, float* out, int64_t ld_out,
                                     int32_t* error_flag, dlrm_stream_t stream);
/* Its backward: the rows re-gathered from `weights` (call before the embedding update);
 * gradients and relu_x as dlrm_interact_dot_backward. */
int dlrm_interact_dot_backward_gather(int32_t B, int32_t F, int32_t D, const float* x,
                                      int64_t x_bstride, const float* weights,
                                      const int64_t* row_base, const int32_t* indices,
                                      int32_t self_interaction, const float* grad_out,
                                      int64_t ld_gout, float* const* grad_ptrs,
                                      const int64_t* grad_bstrides, int32_t relu_x,
                                      dlrm_stream_t stream);
/* Cat: out[b][f*D:(f+1)*D] = feature f. */
int dlrm_interact_cat_forward(int32_t B, int32_t F, int32_t D, const float* const* feat_ptrs,
                              const int64_t* feat_bstrides, float* out, int64_t ld_out,
                              dlrm_stream_t stream);
int dlrm_interact_cat_backward(int32_t B, int32_t F, int32_t D, const float* grad_out,
                               int64_t ld_gout, float* const* grad_ptrs,
                               const int64_t* grad_bstrides, dlrm_stream_t stream);

/* ------------------------------------------------------------------- MLP --- */
/*
 * C[M][N] = epilogue(alpha * op(A)[M][K] . op(B)[K][N]) in exact fp32 on the
 * gfx950 fp32 MFMA (v_mfma_f32_16x16x4_f32), row-major everywhere:
 *   op(A)(m,k) = trans_a ? A[k*lda + m] : A[m*lda + k]
 *   op(B)(k,n) = trans_b ? B[n*ldb + k] : B[k*ldb + n]
 * Linear forward  Y = X W^T + b : trans_a=0, trans_b=1, EPI_BIAS[_RELU]
 * Linear dgrad    dX = dY W     : trans_a=0, trans_b=0, EPI_STORE / EPI_DRELU
 * Linear wgrad    dW = dY^T X   : trans_a=1, trans_b=0, EPI_STORE / EPI_SGD
 * Bias folding: with a constant-1 column appended to X and the bias stored as the
 * matching extra column of W, the forward needs no bias epilogue (EPI_RELU) and the
 * wgrad GEMM produces the bias gradient in that column.
 * Small-M*N / long-K shapes are split along K into >= 2 workgroups per CU when a
 * workspace of dlrm_gemm_f32_workspace_size() bytes is given: the last workgroup of
 * each output tile sums the partials in split order (deterministic) inside the same
 * launch.  The first 64 KiB of the workspace are per-tile tickets that MUST be zero
 * before its first use (hipMemset once); every call leaves them zero again.  Concurrent calls
 * (different streams) need different workspaces.  With workspace == NULL the GEMM runs
 * unsplit.
 */
size_t dlrm_gemm_f32_workspace_size(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N,
                                    int64_t K);
int dlrm_gemm_f32(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K,
                  float alpha, const float* A, int64_t lda, const float* B, int64_t ldb,
                  float* C, int64_t ldc, int32_t epilogue, const float* bias,
                  const float* aux, int64_t ld_aux, void* workspace, size_t workspace_bytes,
                  dlrm_stream_t stream);

/* dlrm_gemm_problem.mode */
enum dlrm_gemm_mode {
  DLRM_GEMM_FULL = 0,    /* C = epilogue(...) (split-K, if planned, reduced in-launch)  */
  DLRM_GEMM_PARTIAL = 1, /* K split `splits` ways; raw partials -> partial buffer:
                            [splits][M][N] (+ [splits][M] row sums for ones_col); no C */
  DLRM_GEMM_REDUCE = 2   /* C = epilogue(alpha * sum_s partial[s]) in split order (+ the
                            ones_col row sums): finishes an earlier PARTIAL problem; a
                            later launch's kernel boundary publishes the partials       */
};

/*
 * Grouped GEMM: up to 6 INDEPENDENT problems in one launch (4 before ABI v5) (e.g. the dgrad of layer l
 * beside the wgrad of layer l+1 of an MLP backward: both read dY_{l+1}, neither writes
 * what the other reads).  Each problem is dlrm_gemm_f32's contract, plus:
 *   ones_col >= 0:  C[m][ones_col] = epilogue(alpha * sum_k op(A)(m,k))   (ones_col in
 *                   [N, ldc)) — the bias gradient of a Linear layer whose bias is stored
 *                   as the weight column ones_col (dW and db of [W | b] in one launch).
 * mode PARTIAL + REDUCE defer a split-K reduction to a LATER launch (typically the next
 * group of an MLP backward, which runs anyway), fully parallel and with no in-launch
 * hand-off; the sum order is fixed (bitwise the in-launch result).  PARTIAL needs
 * aligned operands (K % 4 == 0); REDUCE needs N % 4 == 0; `partial` holds
 * dlrm_gemm_f32_partial_bytes(M, N, splits) bytes.  `splits` = 0 in PARTIAL takes the
 * planner's choice (dlrm_gemm_f32_splits); a PARTIAL count > 0 must already be
 * normalized (dlrm_gemm_f32_splits of the problem with that count returns it unchanged;
 * otherwise INVALID_ARG); REDUCE must repeat the PARTIAL's value.
 * Problems with unaligned operands run on a generic kernel (separate launch, unsplit).
 * The workspace follows dlrm_gemm_f32's rules (zeroed 64 KiB ticket head before first
 * use; one workspace per stream).
 */
typedef struct dlrm_gemm_problem {
  int32_t trans_a, trans_b;
  int64_t M, N, K;
  float alpha;
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  float* C;
  int64_t ldc;
  int32_t epilogue;
  const float* bias;
  const float* aux;
  int64_t ld_aux;
  int64_t ones_col; /* -1: none */
  int32_t mode;     /* dlrm_gemm_mode */
  int32_t splits;   /* PARTIAL / REDUCE */
  float* partial;   /* PARTIAL / REDUCE */
} dlrm_gemm_problem;

size_t dlrm_gemm_f32_group_workspace_size(int32_t n, const dlrm_gemm_problem* problems);
/* The planner's K split for one problem as if launched alone, in its mode (FULL: an
 * in-launch split; PARTIAL: the split a deferred REDUCE will finish).  PARTIAL with
 * splits > 0: that count normalized to K (at most 32 and ceil(K/32); equal chunks of
 * 32-multiples), the count the launch will use. */
int32_t dlrm_gemm_f32_splits(const dlrm_gemm_problem* problem);
size_t dlrm_gemm_f32_partial_bytes(int64_t M, int64_t N, int32_t splits);
int dlrm_gemm_f32_group(int32_t n, const dlrm_gemm_problem* problems, void* workspace,
                        size_t workspace_bytes, dlrm_stream_t stream);
/* dlrm_gemm_f32_group plus pass `phase` of a deferred role as extra workgroups of the same
 * launch: 1 / 2 the embedding update (dlrm_tbe_backward_defer), 4 the head's finalize pass
 * (dlrm_head_step_defer); phase 3 (a deferred per-table sort) was removed in v7; n may be 0
 * (the pass alone).  role == NULL, or a role with nothing deferred: dlrm_gemm_f32_group.  The
 * problems must not touch the update's buffers (weights, momentum, grad_out, workspace). */
int dlrm_gemm_f32_group_role(int32_t n, const dlrm_gemm_problem* problems, void* workspace,
                             size_t workspace_bytes, const dlrm_launch_role* role,
                             int32_t phase, dlrm_stream_t stream);

/* Workspace for dlrm_colsum_f32 (deterministic two-pass column reduction). */
size_t dlrm_colsum_workspace_size(int64_t M, int64_t N);
/*
 * s[n] = sum_m scale[m] * Y[m*ldy + n]   (scale may be NULL == 1), fixed order.
 * If out != NULL: out[n] = alpha * s[n] (or out[n] += alpha*s[n] when accumulate).
 * If sgd_param != NULL: sgd_param[n] -= lr * s[n].
 */
int dlrm_colsum_f32(int64_t M, int64_t N, const float* Y, int64_t ldy, const float* scale,
                    float alpha, float* out, int32_t accumulate, float* sgd_param, float lr,
                    void* workspace, size_t workspace_bytes, dlrm_stream_t stream);

/* Workspace for dlrm_head_forward_backward. */
size_t dlrm_head_workspace_size(int64_t M);
/*
 * Last layer (K -> 1) + sigmoid + mean loss + its gradient, fused:
 *   z[m] = X[m].w + b; p[m] = sigmoid(z[m]); (optional clamp to [lo, 1-lo] when
 *   0 < clamp_lo < 0.5); loss = mean_m l(p_c[m], t[m]) (mse | bce with log >= -100)
 *   dz[m] = grad_scale * dloss/dz[m]
 * prob_out[M], dz_out[M] and *loss_out are device buffers (any may be NULL).
 */
int dlrm_head_forward_backward(int64_t M, int64_t K, const float* X, int64_t ldx,
                               const float* w, const float* b, const float* target,
                               int32_t loss_kind, float clamp_lo, float grad_scale,
                               float* prob_out, float* dz_out, float* loss_out, void* workspace,
                               size_t workspace_bytes, dlrm_stream_t stream);

/* Workspace for dlrm_head_step. */
size_t dlrm_head_step_workspace_size(int64_t M, int64_t K);
/*
 * The whole head of the training step in two launches (bias folded: X carries a
 * constant-1 column and w[K] includes the bias):
 *   z = X w, p = sigmoid(z), loss and dz exactly as dlrm_head_forward_backward;
 *   dX[m][k] = dz[m] * w[k] * (relu_mask ? X[m][k] > 0 : 1)      (if dX != NULL)
 *   s[k] = sum_m dz[m] X[m][k]  (fixed order: 16-row blocks, then blocks in order)
 *   dw_out != NULL: dw_out = s (or += s when accumulate); else if lr != 0: w -= lr * s
 *   (w is updated after every read of it, so dX uses the pre-update weights).
 * K <= 2048.  Replaces head_forward_backward + outer_drelu + colsum for the DLRM head
 * (dlrm_s_pytorch.py:170-178, 504-516, the last Linear of create_mlp).
 */
int dlrm_head_step(int64_t M, int64_t K, const float* X, int64_t ldx, float* w,
                   const float* target, int32_t loss_kind, float clamp_lo, float grad_scale,
                   float* prob_out, float* dz_out, float* loss_out, float* dX, int64_t lddx,
                   int32_t relu_mask, float* dw_out, int32_t accumulate, float lr,
                   void* workspace, size_t workspace_bytes, dlrm_stream_t stream);
/* dlrm_head_step with its second launch (the column sums, the weight update and the mean
 * loss) deferred: *role becomes pass 4 of a later dlrm_gemm_f32_group_role (typically the
 * top-MLP backward's first launch, which reads dX but not w).  The workspace, w, dw_out
 * and loss_out must stay as they are until then; prob_out / dz_out / dX are written here.
 * (ABI v6) */
int dlrm_head_step_defer(int64_t M, int64_t K, const float* X, int64_t ldx, float* w,
                         const float* target, int32_t loss_kind, float clamp_lo,
                         float grad_scale, float* prob_out, float* dz_out, float* loss_out,
                         float* dX, int64_t lddx, int32_t relu_mask, float* dw_out,
                         int32_t accumulate, float lr, void* workspace, size_t workspace_bytes,
                         dlrm_launch_role* role, dlrm_stream_t stream);

/* Elementwise: dX[m][k] = dz[m] * w[k] * (relu_mask ? (X[m][k] > 0) : 1). */
int dlrm_outer_drelu(int64_t M, int64_t K, const float* dz, const float* w, const float* X,
                     int64_t ldx, int32_t relu_mask, float* dX, int64_t lddx,
                     dlrm_stream_t stream);

/* ----------------------------------------------------------- optimizers ---- */
int dlrm_sgd_update(float* param, const float* grad, int64_t n, float lr, dlrm_stream_t stream);
/* state_sum += g^2; param -= clr * g / (sqrt(state_sum) + eps) */
int dlrm_adagrad_update(float* param, const float* grad, float* state_sum, int64_t n, float clr,
                        float eps, dlrm_stream_t stream);
/* The same with the gradient scaled first, g' = grad_scale * g (the several-GPU dense update:
 * the 1/W of the averaged gradient folded in; bitwise dlrm_scale_f32 + dlrm_adagrad_update
 * without the extra pass over the bucket; ABI v9).  Replaces the reference's DDP-averaged
 * RWSAdagrad dense step (optim/rwsadagrad.py:56-122 on dlrm_s_pytorch.py:1626-1633 grads). */
int dlrm_adagrad_update_scaled(float* param, const float* grad, float* state_sum, int64_t n,
                               float grad_scale, float clr, float eps, dlrm_stream_t stream);
int dlrm_scale_f32(float* x, int64_t n, float alpha, dlrm_stream_t stream);

/* Elementwise activations (nn.Sigmoid / nn.ReLU forward & backward on n floats). */
int dlrm_sigmoid_forward(int64_t n, const float* x, float* y, dlrm_stream_t stream);
/* dx = dy * (1 - y) * y */
int dlrm_sigmoid_backward(int64_t n, const float* dy, const float* y, float* dx,
                          dlrm_stream_t stream);
/* dx[m][k] = dy[m][k] * (y[m][k] > 0) over an M x K block of row-strided matrices */
int dlrm_relu_backward(int64_t M, int64_t K, const float* dy, int64_t lddy, const float* y,
                       int64_t ldy, float* dx, int64_t lddx, dlrm_stream_t stream);

/* ------------------------------------------------------------- utilities --- */
/* out[i] = lo + (hi - lo) * u_i, u_i uniform in [0,1) from a counter hash of (seed, i). */
int dlrm_uniform_fill(float* out, int64_t n, float lo, float hi, uint64_t seed,
                      dlrm_stream_t stream);
/* Integer uniform draws in [0, hi) for synthetic indices (int32 or int64 out). */
int dlrm_uniform_int_fill(void* out, int32_t out_bits, int64_t n, int64_t hi, uint64_t seed,
                          dlrm_stream_t stream);

/*
 * Device CSR builder (dlrm_data_pytorch.py:748-753): T per-table offset arrays
 * (each B starts, table-local, first == 0) + per-table index counts ->
 * batched offsets [T*B+1] (int32/int64 by out_offset_bits):
 *   out[t*B + b] = table_start[t] + offsets_t[b], out[T*B] = table_start[T]
 * table_offsets: host array of T device pointers (int64 each, B entries);
 * table_nnz: host int64 [T] (indices per table).
 */
int dlrm_csr_from_tables(int32_t T, int32_t B, const int64_t* const* table_offsets,
                         const int64_t* table_nnz, void* out_offsets, int32_t out_offset_bits,
                         dlrm_stream_t stream);

/*
 * Criteo binary records -> one step's device inputs (replaces the host-side
 * CriteoBinDataset.__getitem__ -> _transform_features, data_loader_terabyte.py:237-252,
 * 83-114).  `records` is the raw int32 block [n][1 + n_dense + n_sparse] of the binary
 * file written by numpy_to_binary (:255-293), already on the device.  Writes
 *   label[n]                       = (float)label           (may be NULL)
 *   dense[b * ld_dense + j]        = log((float)x_int + 1)  (may be NULL)
 *   indices[t * n + b]             = x_cat[b][t] mod max_ind_range (floor mod, as torch
 *                                    `%`; no mod when max_ind_range <= 0), table-major
 *                                    = cat(x_cat.t()); index_bits 32 (batched) or 64
 *   offsets[i] = i, i <= n_sparse*n  (table-batched CSR, L = 1; may be NULL)
 * Integer outputs are bit-exact; the dense log is fp32.
 */
int dlrm_criteo_decode(const int32_t* records, int64_t n, int32_t n_dense, int32_t n_sparse,
                       int64_t max_ind_range, float* dense, int64_t ld_dense, float* label,
                       void* indices, int32_t index_bits, void* offsets, int32_t offset_bits,
                       dlrm_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DLRM_HIP_H_ */
