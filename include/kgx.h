/*
 * kgx.h — C-ABI of the MI355X-native message-passing aggregation engine.
 *
 * This is the drop-in boundary for keras-geometric's MessagePassing.propagate()
 * hot path (edge-index gather -> message -> segment-{sum,mean,max,min,std}
 * scatter).  Every entry point takes plain device pointers, sizes and a HIP
 * stream (passed as an opaque pointer so callers need no HIP headers), returns
 * an int status (KGX_OK == 0) and never allocates or frees memory: buffers are
 * owned by the caller (the torch caching allocator in the Python host layer).
 * On failure kgx_last_error() returns a thread-local message.
 *
 * Reference citations are relative to the keras-geometric snapshot the survey
 * studied (src/keras_geometric/...).  The reference itself is pure Python on
 * Keras-3 ops; each function below names the reference code it replaces.
 *
 * Conventions
 *   - node features are fp32, row-major, leading dimension `ld_*` in elements;
 *   - edge ids / node ids are int32 (the reference casts edge_index to int32:
 *     layers/message_passing.py:265, layers/gcn_conv.py:307);
 *   - E (edges) must be < 2^31 - n_dst; feature offsets are computed in int64.
 */
#ifndef KGX_H_
#define KGX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* kgx_stream_t; /* a hipStream_t; NULL = the null stream */

enum kgx_status {
  KGX_OK = 0,
  KGX_ERR_ARG = 1,         /* bad sizes / null pointers / misalignment      */
  KGX_ERR_HIP = 2,         /* HIP runtime error (launch, memcpy, ...)        */
  KGX_ERR_INDEX = 3,       /* an edge index lies outside the node range      */
  KGX_ERR_UNSUPPORTED = 4  /* shape the kernels do not implement             */
};

/* Segment reductions: layers/aggregators.py Sum(:119-141) Mean(:48-89)
 * Max(:92-116) Min(:144-171) Std(:174-232).                                  */
enum kgx_reduce { KGX_SUM = 0, KGX_MEAN = 1, KGX_MAX = 2, KGX_MIN = 3, KGX_STD = 4 };

/* Fused epilogues applied after the reduction of a destination row.
 *   BIAS: out = aggr + bias[f]              (GCNConv.update, gcn_conv.py:266-272)
 *   GIN : out = gin_scale * x[row,f] + aggr (GINConv.update, gin_conv.py:216-222)
 *   RAW : MAX / MIN without the aggregators' isinf -> 0 guard: plain
 *         keras.ops.segment_max semantics (empty segment -> -inf), as
 *         BatchGlobalPooling uses it (global_pooling.py:228-249)            */
/* KGX_EPI_ACCUM (reduce KGX_SUM only): out[row] += this launch's row sum, read
 * from and written to `out` in place -- the sharded GIN / SAGE halo-chunk
 * passes (no reference counterpart; distributed.py). */
enum kgx_epilogue { KGX_EPI_NONE = 0, KGX_EPI_BIAS = 1, KGX_EPI_GIN = 2, KGX_EPI_RAW = 3, KGX_EPI_ACCUM = 4 };

/* Graph-preparation flags. */
enum kgx_csr_flags {
  KGX_CSR_SELF_LOOPS = 1, /* append (i,i) after the E input edges: utils/main.py:8-16    */
  KGX_CSR_SEGMENT_ONLY = 2, /* segment semantics only (Aggregator.aggregate called directly,
                               aggregators.py:24-39): ids outside [0,n_dst) are dropped,
                               src is not validated                                       */
  KGX_CSR_GCN_NORM = 4    /* also produce dinv[n_dst] and per-CSR-edge weight w:
                               utils/main.py:20-33                                        */
};

int kgx_version(void);
const char* kgx_last_error(void);

/* ---------------------------------------------------------------------------
 * The CU split (KGX_FUSED_CU_SPLIT launches): validated on gfx950 with 256 CUs
 * in 8 XCDs only.  kgx_cu_split_layout_ok: 1 when (cus, xccs, arch) is that
 * layout (pure, no device needed).  kgx_cu_split_supported: 1 when `device`
 * has it, 0 when its KGX_FUSED_CU_SPLIT launches run unsplit (one note on
 * stderr), < 0 on error.  A launch whose stream is on another device than the
 * current one also runs unsplit.
 * ------------------------------------------------------------------------- */
int kgx_cu_split_layout_ok(int cus, int xccs, const char* arch);
int kgx_cu_split_supported(int device);
/* Census of the CU-masked streams a split launch uses (a diagnostic the tests run):
 * n_blocks short blocks on the head stream and n_blocks on the tail stream of
 * cu_split(per32) each record where they ran, (XCC id << 8) | (SE id << 5) |
 * (SH id << 4) | CU id from the hardware registers, into head_ids[n_blocks] and
 * tail_ids[n_blocks]; n_cus[0] / n_cus[1] = the head / tail CU counts the split
 * believes its masks hold.  Synchronises the caller's stream.  KGX_ERR_UNSUPPORTED
 * when the device has no validated split layout.  Checks that the masks are
 * disjoint and cover what they claim (tests/test_gpu_cu_census.py). */
int kgx_cu_split_census(int per32, int64_t n_blocks, int32_t* head_ids, int32_t* tail_ids, int* n_cus,
                        kgx_stream_t stream);

/* ---------------------------------------------------------------------------
 * Graph preparation: COO int32 [2,E] (generation order, unsorted) -> CSR by
 * destination, STABLE (edges of one destination keep their input order, the
 * self-loop is last), which is the order the reference's segment_sum
 * (Keras-torch scatter_add) accumulates in.
 *
 * Replaces: MessagePassing.call edge_index cast/cache (message_passing.py:256-268),
 *           add_self_loops (utils/main.py:8-16), the degree segment_sum of
 *           compute_gcn_normalization (utils/main.py:23-24) and of
 *           MeanAggregator (aggregators.py:66-69).
 *
 * Index semantics (Keras-3 torch lowering of take/segment_sum):
 *   src in [-n_src, n_src): negative ids wrap (+n_src), else KGX_ERR_INDEX;
 *   dst in [-n_dst, n_dst): negative ids are dropped from every segment
 *   reduction (and from degrees), else KGX_ERR_INDEX.
 *   With KGX_CSR_SEGMENT_ONLY every dst outside [0,n_dst) is dropped.
 * Outputs (caller-allocated, capacity E + n_dst when SELF_LOOPS else E):
 *   rowptr[n_dst+1], col[cap] (source id per CSR slot), eid[cap] (input edge
 *   id per CSR slot; self loop i has id E+i), deg[n_dst] (int32 in-degree),
 *   optional dinv[n_dst] and w[cap] (KGX_CSR_GCN_NORM).
 * info[4] (host) receives: kept edges, max in-degree, #bad indices, and
 * (kgx_csr_build2) the rows whose degree the dinv table did not cover.
 * This call synchronises `stream` once (to return info).
 *
 * GCN_NORM's dinv: kgx_csr_build computes (deg + 1e-12)^-0.5 correctly
 * rounded.  kgx_csr_build2 takes it from the caller's device table instead,
 *   dinv[i] = dinv_table[min(deg[i], 2^24)],   table_len entries,
 * filled with the reference's own values: utils/main.py:25's
 * power(deg + 1e-12, -0.5) lowers to torch.pow(Tensor, Tensor), ATen's
 * vectorised (Sleef) powf, which differs from the correctly-rounded value by
 * 1 ulp for some degrees.  With that table dinv and w are bit-identical to
 * the reference's (graph.gcn_dinv_table builds it).  A degree the table does
 * not cover takes the correctly-rounded value and is counted in info[3]; the
 * caller then redoes dinv / w with a longer table (kgx_gcn_dinv_table +
 * kgx_gcn_edge_norm).  dinv_table NULL: kgx_csr_build.
 * ------------------------------------------------------------------------- */
int kgx_csr_workspace_bytes(int64_t E, int64_t n_dst, int flags, size_t* bytes);
int kgx_csr_build(const int32_t* src, const int32_t* dst, int64_t E,
                  int64_t n_src, int64_t n_dst, int flags,
                  int32_t* rowptr, int32_t* col, int32_t* eid, int32_t* deg,
                  float* dinv, float* w,
                  void* workspace, size_t workspace_bytes,
                  int64_t* info, kgx_stream_t stream);
int kgx_csr_build2(const int32_t* src, const int32_t* dst, int64_t E,
                   int64_t n_src, int64_t n_dst, int flags,
                   int32_t* rowptr, int32_t* col, int32_t* eid, int32_t* deg,
                   float* dinv, float* w, const float* dinv_table, int64_t table_len,
                   void* workspace, size_t workspace_bytes,
                   int64_t* info, kgx_stream_t stream);

/* ---------------------------------------------------------------------------
 * Schedule tails, on the device (the fused kernels' short-row and tiny-row
 * launches take the degree-descending schedule's suffix of small unsplit rows):
 * kgx_schedule_suffixes: out[0] = 1 + the last item (int4 {row, beg, end,
 * slot}) that is split or has more than short_max edges, out[1] the same for
 * tiny_max (0: none).  kgx_tiny_pack: the records of items [start, start+n):
 * pack[i] = {row, degree, col0, col1} (col1 = col0 for degree 1, 0 / 0 for
 * degree 0; indices clamped to n_col - 1), tw[i] = {w0, w1} (0 where absent;
 * tw NULL: unweighted); out[0] = records of degree 2, out[1] = 1 + the last
 * of them.  Both take a 16-byte device workspace and synchronise `stream`.
 * ------------------------------------------------------------------------- */
int kgx_schedule_suffixes(const int32_t* items, int64_t n_items, int short_max, int tiny_max,
                          void* workspace, int64_t* out, kgx_stream_t stream);
int kgx_tiny_pack(const int32_t* items, int64_t start, int64_t n, const int32_t* col, const float* w,
                  int64_t n_col, int32_t* pack, float* tw, void* workspace, int64_t* out,
                  kgx_stream_t stream);

/* ---------------------------------------------------------------------------
 * GCN normalisation for a CSR whose sources index a different table than its
 * rows (a destination-range shard: rows = owned nodes, sources = owned + halo
 * nodes).  Same arithmetic as KGX_CSR_GCN_NORM (utils/main.py:20-33):
 *   dinv[i] = (float(min(deg[i], 2^24)) + 1e-12f)^-0.5  (correctly rounded)
 *   w[e]    = dinv_dst[row(e)] * dinv_src[col[e]]       (CSR order)
 * kgx_gcn_dinv_table: dinv[i] = table[min(deg[i], 2^24)] (the reference's
 * values, see kgx_csr_build2); the caller's table must cover
 * min(max(deg), 2^24) (indices past it read the last entry).
 * ------------------------------------------------------------------------- */
int kgx_gcn_dinv(const int32_t* deg, int64_t n, float* dinv, kgx_stream_t stream);
int kgx_gcn_dinv_table(const int32_t* deg, int64_t n, const float* table, int64_t table_len,
                       float* dinv, kgx_stream_t stream);
int kgx_gcn_edge_norm(const int32_t* rowptr, const int32_t* col, int64_t n_dst,
                      const float* dinv_dst, const float* dinv_src, float* w,
                      kgx_stream_t stream);

/* ---------------------------------------------------------------------------
 * Row schedule (no reference counterpart: the reference has one device and no
 * scheduling).  Orders destination rows by descending degree (log2 buckets,
 * stable) so hub rows start first, and cuts rows with deg >= split_len into
 * split_len-edge chunks whose partials are combined in chunk order.
 *   rows[n_dst]              row ids in schedule order (EXACT mode iterates these)
 *   items[4*cap_items]       {row, edge_begin, edge_end, partial_slot|-1}
 *   split[4*n_dst]           {row, first_slot, n_chunks, degree} for split rows
 * cap_items must be >= n_dst + E_kept / split_len + 1.  split_len <= 0 means
 * never split.  info[4] (host): n_items, n_split_rows, n_slots, 0.  Syncs once.
 * ------------------------------------------------------------------------- */
int kgx_schedule_workspace_bytes(int64_t n_dst, size_t* bytes);
int kgx_schedule_build(const int32_t* rowptr, int64_t n_dst, int32_t split_len,
                       int32_t* rows, int32_t* items, int64_t cap_items,
                       int32_t* split, void* workspace, size_t workspace_bytes,
                       int64_t* info, kgx_stream_t stream);

/* ---------------------------------------------------------------------------
 * Fused gather -> (weight) -> segment reduction -> epilogue, one launch.
 *   out[row, f] = EPI( REDUCE_{e in CSR row} table[idx[e], f] * (w ? w[e] : 1) )
 *
 * Replaces: MessagePassing.propagate's take(x_j, src) (message_passing.py:195),
 *   the default/GCN/GIN/SAGE message (message_passing.py:73-77, gcn_conv.py:233-248,
 *   gin_conv.py:193, sage_conv.py:294-298), MessagePassing.aggregate ->
 *   Aggregator.aggregate (message_passing.py:79-102, aggregators.py:48-232) and
 *   the GCN/GIN update epilogues.
 * With idx = col and table = node features it is the node-gather SpMM; with
 *   idx = eid and table = a per-edge message tensor [E,F] it is the reference's
 *   Aggregator.aggregate(messages, target_idx, dim_size) on arbitrary messages.
 * Work list: if items != NULL the (possibly split) item list of
 *   kgx_schedule_build is used and split rows are finished by an in-call fix-up
 *   (partials: n_slots*F floats); otherwise every row of `rows` is reduced
 *   sequentially in CSR order (EXACT: bit-identical to the reference's
 *   sequential scatter_add / scatter_reduce for identical messages).
 * KGX_STD ignores items (always EXACT, two sequential passes per row).
 * drop_key (optional, SUM only): per-slot keys of the message dropout mask
 * (see kgx_dropout_mask); the message is (table[idx] * mask) * w.
 * ------------------------------------------------------------------------- */
int kgx_spmm(int reduce, int epilogue,
             const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
             const int32_t* items, int64_t n_items,
             const int32_t* split, int64_t n_split,
             const int32_t* idx, const float* w,
             const float* table, int64_t ld_table, int64_t F,
             float* out, int64_t ld_out,
             const float* bias, const float* xroot, int64_t ld_x, float gin_scale,
             const int32_t* drop_key, float drop_p, uint64_t drop_seed,
             float* partials, kgx_stream_t stream);
/* kgx_spmm with the schedule's short-row suffix named: items [n_long_items,
 * n_items) are unsplit rows of degree <= KGX_SHORT_ROW_MAX (defined below),
 * taken several per lane group by a second kernel (not with message dropout
 * or column slices wider than 64 lanes).  n_long_items = n_items is kgx_spmm.
 * EXACT mode (items = NULL): 0 < n_long_items < n_rows names the same suffix
 * of the degree-descending `rows` list, rows[n_long_items, n_rows), for the
 * same kernel (each row still one chain of adds in CSR order: bit-identical);
 * any other value leaves every row to the main kernel. */
int kgx_spmm_ex(int reduce, int epilogue, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                const int32_t* items, int64_t n_items, int64_t n_long_items, const int32_t* split,
                int64_t n_split, const int32_t* idx, const float* w, const float* table, int64_t ld_table,
                int64_t F, float* out, int64_t ld_out, const float* bias, const float* xroot, int64_t ld_x,
                float gin_scale, const int32_t* drop_key, float drop_p, uint64_t drop_seed, float* partials,
                kgx_stream_t stream);

/* kgx_spmm_ex2: kgx_spmm_ex gathering from TWO tables: sources c < n_table1 are
 * rows of table, c >= n_table1 rows c - n_table1 of table2 (same ld_table).
 * Needs the schedule (items; not EXACT / std).  The sharded GIN / SAGE layers
 * reduce a row's own-source and halo edges in one pass (distributed.py).
 * table2 NULL: kgx_spmm_ex.
 * counters (EXACT mode, items NULL): two caller-owned int32, zeroed before the
 * call, from which the hub-row kernel (rows of >= 2048 edges) hands out its
 * (row, column group) items dynamically, so its blocks balance instead of
 * waiting behind the largest row (bit-identical results: every row is still
 * reduced by one lane chain in CSR order, aggregators.py:126-137).  NULL: the
 * static schedule.  With counters the hub kernel also forks onto a
 * library-owned stream beside the main kernel (joined back into `stream`
 * before the call returns), and the main kernel takes interleaved batches of
 * rows from counters[1] (batch b = rows b, b + NB, ..., one atomic per 8 rows),
 * so the GPU is not idle behind the largest hub row (KGX_EXACT_FORK=0: the
 * sequential form). */
int kgx_spmm_ex2(int reduce, int epilogue, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                 const int32_t* items, int64_t n_items, int64_t n_long_items, const int32_t* split, int64_t n_split,
                 const int32_t* idx, const float* w, const float* table, int64_t ld_table, const float* table2,
                 int64_t n_table1, int64_t F, float* out, int64_t ld_out, const float* bias, const float* xroot,
                 int64_t ld_x, float gin_scale, const int32_t* drop_key, float drop_p, uint64_t drop_seed,
                 float* partials, int32_t* counters, kgx_stream_t stream);

/* Message dropout mask (training; GCNConv.message dropout, gcn_conv.py:237-242;
 * GATv2 attention dropout, gatv2_conv.py:252-253): element (key, f) is kept
 * with probability 1 - p and scaled by 1/(1-p).  The mask is a pure function
 * of (seed, key = input edge id, f), so a layer's forward (kgx_spmm with
 * drop_key = the CSR's input edge ids), its backward over the transposed
 * graph and tests agree.  kgx_dropout_mask writes the multiplier (0 or
 * 1/(1-p)) of n keys x F columns, row-major. */
int kgx_dropout_mask(uint64_t seed, float p, const int32_t* keys, int64_t n, int64_t F, float* out,
                     kgx_stream_t stream);

/* ---------------------------------------------------------------------------
 * Fused aggregate -> dense transform (+ bias), one launch (plus a fix-up for
 * split hub rows):
 *   out[i,:] (+)= bias + PRE( REDUCE_{e in row i} x[idx[e],:] * (w ? w[e] : 1) ) @ W
 *   PRE = identity, or gin_scale * x[i,:] + aggr with KGX_FUSED_PRE_GIN;
 *   "+=" (read-add-write of out) with KGX_FUSED_ACCUMULATE, used to add the
 *   halo-source part of a sharded row after its local part (distributed.py),
 *   and SAGEConv's neighbour map onto out = b + x W_self (sage_conv.py:404-433).
 * Replaces GCNConv's per-edge x_j @ W + segment_sum + bias (gcn_conv.py:233-272)
 * and GINConv's (1+eps)x + aggr -> single-Dense MLP (gin_conv.py:216-225) by the
 * algebraically equal aggregate-then-transform order (W applied once per row
 * on MFMA as the six significant products of a three-way bf16 split of both
 * operands: f32-accurate); tolerance-equal to the reference, not bit-equal.
 * Shapes: F_in and F_out multiples of 4 <= 128, W [F_in, F_out] row-major.
 * reduce in {SUM, MEAN, MAX, MIN}; partials: n_slots * 128 floats.
 * agg_out (optional, [n, ld_agg >= F_in]): also store PRE(REDUCE(...)), the
 * rows before the transform — what the backward's dW = agg^T dOut needs.
 * ------------------------------------------------------------------------- */
/* KGX_FUSED_SHARE_GPU: launch (den - 1) / den of the resident grid (den =
 * KGX_SHARE_DEN, default 16; the 256-wide kernels take the flag and ignore it), leaving block slots
 * for kernels of a concurrent stream (the sharded layer's RCCL exchange).
 * KGX_FUSED_RELU: out = max(bias + ..., 0), the activation of a GIN MLP's
 * first Dense (gin_conv.py:129-162) or SAGEConv's activation; with ACCUMULATE
 * it applies to the sum (out = max(out + ..., 0)).  kgx_spmm_gemm_f256 rejects
 * RELU | ACCUMULATE. */
/* KGX_FUSED_CU_SPLIT: run the schedule's tail launches on a CU-masked stream
 * over 8 of every 32 CUs, beside the main launches on the other CUs; both
 * streams are forked from and joined back into `stream` (before the hub
 * fix-up).  Outputs are bit-identical to the one-stream order.
 * kgx_spmm_gemm_f256 / _f256_ex: the tail is the degree <= 2 records (MFMA-
 * bound), the main part the long rows and degree 3..7 (memory-bound);
 * KGX_F256_CU_SPLIT (environment) = tail CUs per 32, 0 = ignore the flag.
 * kgx_spmm_gemm*: the tail is the short-row and tiny-record launches, the main
 * part spmm_gemm_kernel; KGX_FUSED_CU_SPLIT (environment) = tail CUs per 32. */
enum { KGX_FUSED_PRE_GIN = 1, KGX_FUSED_ACCUMULATE = 2, KGX_FUSED_SHARE_GPU = 4, KGX_FUSED_RELU = 8,
       KGX_FUSED_CU_SPLIT = 16 };
int kgx_spmm_gemm(int reduce, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                  const int32_t* items, int64_t n_items, const int32_t* split, int64_t n_split,
                  const int32_t* idx, const float* w, const float* x, int64_t ld_x, int64_t F_in,
                  const float* W, int64_t F_out, const float* bias, int flags, float gin_scale,
                  float* out, int64_t ld_out, float* partials, float* agg_out, int64_t ld_agg,
                  kgx_stream_t stream);
/* kgx_spmm_gemm with the schedule's short-row suffix named: items
 * [n_long_items, n_items) are rows of degree <= KGX_SHORT_ROW_MAX (the degree-ordered
 * schedule's tail, never split), reduced 64 rows per block iteration by a
 * second kernel.  n_long_items = n_items is kgx_spmm_gemm. */
enum { KGX_SHORT_ROW_MAX = 7 };
int kgx_spmm_gemm_ex(int reduce, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                     const int32_t* items, int64_t n_items, int64_t n_long_items, const int32_t* split,
                     int64_t n_split, const int32_t* idx, const float* w, const float* x, int64_t ld_x,
                     int64_t F_in, const float* W, int64_t F_out, const float* bias, int flags,
                     float gin_scale, float* out, int64_t ld_out, float* partials, float* agg_out,
                     int64_t ld_agg, kgx_stream_t stream);

/* kgx_spmm_gemm_ex2: kgx_spmm_gemm_ex with the schedule's tail of rows of degree
 * <= 2 ([n_short_end, n_items)) taken from packed records instead of the item
 * list: tiny_pack[n_items - n_short_end][4] = {row, degree, col0, col1} (col1 =
 * col0 for degree 1, both any valid source for degree 0) and, when w is given,
 * tiny_w[..][2] = {w0, w1}; the first n_tiny_deg2 records have degree 2 (the
 * rest <= 1: degree-descending order).  Built once per graph (tiny.py).  Items
 * [n_long_items, n_short_end) go to the short-row kernel as before.  tiny_pack
 * NULL: n_short_end must equal n_items.  Same boundary as kgx_spmm_gemm
 * (gcn_conv.py:233-272, aggregators.py:56-167). */
int kgx_spmm_gemm_ex2(int reduce, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                      const int32_t* items, int64_t n_items, int64_t n_long_items, int64_t n_short_end,
                      const int32_t* tiny_pack, const float* tiny_w, int64_t n_tiny_deg2,
                      const int32_t* split, int64_t n_split,
                      const int32_t* idx, const float* w, const float* x, int64_t ld_x, int64_t F_in,
                      const float* W, int64_t F_out, const float* bias, int flags, float gin_scale, float* out,
                      int64_t ld_out, float* partials, float* agg_out, int64_t ld_agg, kgx_stream_t stream);

/* kgx_spmm_gemm_ex3: kgx_spmm_gemm_ex2 gathering from TWO feature tables:
 * source columns c < n_x1 are rows of x, columns c >= n_x1 are rows
 * c - n_x1 of x2 (same leading dimension ld_x, 16-byte aligned).  The sharded
 * layers' halo pass reads a row's own-source edges from the layer input and
 * its halo edges from the exchange's receive buffer in ONE pass, so the row is
 * written once instead of written and read-modify-written (distributed.py;
 * gcn_conv.py:233-272, gin_conv.py:216-225 per shard).  With x2: sums only
 * (weighted or not, GIN's pre-scale allowed), F_in 128, F_out % 16 == 0.
 * x2 NULL: kgx_spmm_gemm_ex2.  Rows indexed by pre_gin are rows of x. */
int kgx_spmm_gemm_ex3(int reduce, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                      const int32_t* items, int64_t n_items, int64_t n_long_items, int64_t n_short_end,
                      const int32_t* tiny_pack, const float* tiny_w, int64_t n_tiny_deg2,
                      const int32_t* split, int64_t n_split, const int32_t* idx, const float* w,
                      const float* x, int64_t ld_x, const float* x2, int64_t n_x1, int64_t F_in,
                      const float* W, int64_t F_out, const float* bias, int flags, float gin_scale, float* out,
                      int64_t ld_out, float* partials, float* agg_out, int64_t ld_agg, kgx_stream_t stream);

/* kgx_spmm_gemm_f256: kgx_spmm_gemm for 256-wide rows (F_in == 256, F_out a
 * multiple of 16 <= 256; partials n_slots * 256 floats).  GINConv's
 * (1+eps) x + aggr -> Dense at BASELINE config C4 (gin_conv.py:216-225,
 * 129-162) and GCNConv 256 -> 256 (gcn_conv.py:233-272) without the [N, 256]
 * aggregate written and read back.  Items [0, n_short_end) go to the main
 * kernel (as two launches when 0 <= n_long_items < n_short_end: the hub chunks
 * and rows of degree > KGX_SHORT_ROW_MAX first, then the rows of degree <=
 * KGX_SHORT_ROW_MAX, gathered whole a tile ahead; -1: one launch); with tiny_pack, the schedule's tail [n_short_end, n_items) of rows of
 * degree <= 2 comes from the packed records of kgx_spmm_gemm_ex2 (tiny_pack
 * NULL: n_short_end must equal n_items).  One feature table; same flags,
 * argument meaning and error behaviour as kgx_spmm_gemm. */
int kgx_spmm_gemm_f256(int reduce, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                       const int32_t* items, int64_t n_items, int64_t n_long_items, int64_t n_short_end,
                       const int32_t* tiny_pack, const float* tiny_w, const int32_t* split, int64_t n_split,
                       const int32_t* idx, const float* w, const float* x, int64_t ld_x, int64_t F_in,
                       const float* W, int64_t F_out, const float* bias, int flags, float gin_scale,
                       float* out, int64_t ld_out, float* partials, float* agg_out, int64_t ld_agg,
                       kgx_stream_t stream);

/* kgx_spmm_gemm_f256_ex: kgx_spmm_gemm_f256 gathering from TWO feature tables,
 * as kgx_spmm_gemm_ex3: source columns c < n_x1 are rows of x, c >= n_x1 rows
 * c - n_x1 of x2 (same ld_x, 16-byte aligned); pre_gin's root rows are rows of
 * x.  The sharded GINConv's merged halo pass at C4: a row's own-source and
 * halo edges in one launch, (1+eps) x_i + aggr -> Dense, the row written once
 * (distributed.py; gin_conv.py:216-225 per shard).  Sum only with x2; x2 NULL:
 * kgx_spmm_gemm_f256. */
int kgx_spmm_gemm_f256_ex(int reduce, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                          const int32_t* items, int64_t n_items, int64_t n_long_items, int64_t n_short_end,
                          const int32_t* tiny_pack, const float* tiny_w, const int32_t* split, int64_t n_split,
                          const int32_t* idx, const float* w, const float* x, int64_t ld_x, const float* x2,
                          int64_t n_x1, int64_t F_in, const float* W, int64_t F_out, const float* bias, int flags,
                          float gin_scale, float* out, int64_t ld_out, float* partials, float* agg_out,
                          int64_t ld_agg, kgx_stream_t stream);

/* ---------------------------------------------------------------------------
 * Weight and bias gradients of a layer out = P W + b (the fused layers'
 * training step, kgx_dense's backward):
 *   dW[k, m] = sum_n P[n, k] D[n, m]  (K x M, row stride ld_dw)
 *   db[m]    = sum_n D[n, m]          (NULL: not computed)
 * in one pass over P [N, K] and D = dOut [N, M] (row strides ldp, ldd, unit
 * column stride).  bf16x3-split MFMA products (f32-accurate), the node sum
 * split over row ranges and the partials added in a fixed order
 * (deterministic).  A row range holding an inf / NaN is recomputed in plain
 * f32 (IEEE propagation).  Workspace: kgx_gemm_tn_workspace_bytes.
 * Replaces: the reference autograd's matmul / sum backward of
 * gcn_conv.py:233-272 (x_j W, + bias) and of keras Dense (gin_conv.py:129-162,
 * sage_conv.py:404-433).
 * ------------------------------------------------------------------------- */
int kgx_gemm_tn_workspace_bytes(int64_t N, int64_t K, int64_t M, size_t* bytes);
int kgx_gemm_tn(int64_t N, const float* P, int64_t ldp, int64_t K, const float* D, int64_t ldd, int64_t M,
                float* dW, int64_t ld_dw, float* db, void* workspace, size_t workspace_bytes,
                kgx_stream_t stream);

/* ---------------------------------------------------------------------------
 * Backward of the segment max / min reduction (autograd of kgx_spmm MAX/MIN).
 * torch's scatter_reduce amax/amin backward, under the reference's isinf
 * guard (aggregators.py:99-112, 151-167): grad_out[i,f] is shared evenly by
 * the edges of row i whose message equals the row's raw extreme; rows whose
 * extreme is +-inf (empty rows included) or NaN pass nothing.
 *   grad_table[idx[e], f] += grad_out[i, f] / ties   (float atomics)
 * raw != 0 (KGX_EPI_RAW forward): no guard -- a +-inf extreme shares its
 * gradient with its tied edges, and a -inf extreme also with the -inf init
 * (torch's include_self count).
 * grad_table must be zero-initialised by the caller.  Sum / mean / weighted
 * sums need no separate entry point: their backward is kgx_spmm over the
 * transposed graph (a kgx_csr_build of the reversed edges).
 * ------------------------------------------------------------------------- */
int kgx_spmm_max_backward(int reduce, int raw, const int32_t* rowptr, int64_t n_rows, const int32_t* idx,
                          const float* table, int64_t ld_table, int64_t F,
                          const float* grad_out, int64_t ld_grad_out,
                          float* grad_table, int64_t ld_grad_table, kgx_stream_t stream);

/* ---------------------------------------------------------------------------
 * Fused GATv2 attention aggregation (single pass, online segment softmax).
 *   s[e,h]  = sum_c att[h,c] * leaky_relu(h_dst[i,h,c] + h_src[j,h,c], slope)
 *   alpha   = exp(s - max_i) / (sum_i exp(s - max_i) + 1e-10)
 *   out[i,h,c] = sum_e alpha[e,h] * h_src[j,h,c]  (+ bias[h*C+c] if bias)
 * Replaces GATv2Conv._gatv2_propagate's gathers, _compute_attention,
 *   _softmax_by_target, alpha*h_j, _aggregate_messages and the concat-mode
 *   _final_update (gatv2_conv.py:241-266, 268-311, 313-335, 337-352).
 * h_src/h_dst: [n, heads*channels] row-major with leading dimension ld_h.
 * partials: n_slots * (heads*channels + 2*heads) floats when items are split.
 * stats (optional, [n, 2*heads]): per row and head the softmax max and
 * denominator (sum + 1e-10), kept for kgx_gatv2_backward.
 * drop_key (optional): attention dropout (training, gatv2_conv.py:252-253):
 * alpha of (slot e, head h) is multiplied by the kgx_dropout_mask value of
 * (seed, drop_key[e], h); the denominator is not.
 * ------------------------------------------------------------------------- */
int kgx_gatv2(const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
              const int32_t* items, int64_t n_items,
              const int32_t* split, int64_t n_split,
              const int32_t* col, const float* h_src, const float* h_dst, int64_t ld_h,
              const float* att, int heads, int channels, float negative_slope,
              float* out, int64_t ld_out, const float* bias,
              float* partials, float* stats,
              const int32_t* drop_key, float drop_p, uint64_t drop_seed, kgx_stream_t stream);

/* ---------------------------------------------------------------------------
 * Backward of kgx_gatv2 (autograd of GATv2Conv's propagate, gatv2_conv.py:
 * 241-352).  Needs the forward's output `out` (bias included when bias is
 * given) and its per-row softmax `stats` ([n, 2*heads]: max, denominator;
 * kgx_gatv2's optional last output).  Given G = d loss / d out, writes
 * d h_dst (destination CSR + its schedule; split rows via partials), d h_src
 * (pulled over the TRANSPOSED graph: t_rowptr/t_rows/t_items/t_split over
 * sources, t_col = destination row, t_slot = forward CSR slot of each
 * transposed slot), and ADDS d att (grad_att zeroed by the caller).
 * alpha_ws / ds_ws: E' * heads floats of workspace; partials:
 * max(n_slots, t_n_slots) * heads*channels floats.  The bias gradient is a
 * column sum the caller takes.
 * ------------------------------------------------------------------------- */
int kgx_gatv2_backward(const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                       const int32_t* items, int64_t n_items, const int32_t* split, int64_t n_split,
                       const int32_t* col, const float* h_src, const float* h_dst, int64_t ld_h,
                       const float* att, int heads, int channels, float negative_slope,
                       const float* out, int64_t ld_out, const float* bias, const float* stats,
                       const float* grad_out, int64_t ld_grad,
                       const int32_t* t_rowptr, const int32_t* t_rows, int64_t n_src,
                       const int32_t* t_items, int64_t t_n_items, const int32_t* t_split, int64_t t_n_split,
                       const int32_t* t_col, const int32_t* t_slot,
                       float* grad_h_src, float* grad_h_dst, int64_t ld_grad_h, float* grad_att,
                       float* alpha_ws, float* ds_ws, float* partials,
                       const int32_t* drop_key, float drop_p, uint64_t drop_seed, kgx_stream_t stream);

/* ---------------------------------------------------------------------------
 * Dense node transform (the layers' keras Dense / ops.matmul), one launch:
 *   out[i,:] (+)= ACT( bias + x0[i,:K0] @ W0 + x1[i,:K1] @ W1 )
 * Replaces GINConv's MLP Dense (gin_conv.py:129-162, applied at :225),
 * SAGEConv's lin_self(x) + lin_neigh(aggr) + bias (sage_conv.py:407-428: both
 * terms in ONE pass), GATv2Conv's shared linear map (gatv2_conv.py:224-239) and
 * GCNConv's x @ kernel (gcn_conv.py:233-235) where the fused kernel does not
 * apply.  f32-accurate: the product runs on bf16 MFMA as the six significant
 * cross products of a three-way bf16 split of both operands (dropped terms
 * <= 2^-24 |x w|); tolerance-equal to fp32 GEMM, not bit-equal.
 * Shapes: K0 + K1 <= KGX_DENSE_MAX_K, N <= KGX_DENSE_MAX_N, K0 and K1
 * multiples of 4, x rows 16-byte aligned with ld % 4 == 0; W0 [K0, N] and
 * W1 [K1, N] row-major contiguous; x1/W1 may be NULL with K1 = 0; bias [N] or
 * NULL.  KGX_DENSE_RELU: out = max(., 0) (Dense(activation='relu'));
 * KGX_DENSE_ACCUMULATE: out += (before RELU).
 * ------------------------------------------------------------------------- */
enum { KGX_DENSE_RELU = 1, KGX_DENSE_ACCUMULATE = 2 };
enum { KGX_DENSE_MAX_K = 256, KGX_DENSE_MAX_N = 256 };
int kgx_dense(int64_t M, const float* x0, int64_t ld_x0, int64_t K0, const float* W0,
              const float* x1, int64_t ld_x1, int64_t K1, const float* W1, int64_t N,
              const float* bias, int flags, float* out, int64_t ld_out, kgx_stream_t stream);

/* ---------------------------------------------------------------------------
 * Row gather out[i,:] = table[rows[i], :] — packs halo rows for the multi-GPU
 * exchange (no reference counterpart; the reference is single-device) and
 * scatters per-edge values back to input edge order.
 * ------------------------------------------------------------------------- */
int kgx_gather_rows(const float* table, int64_t ld_table, const int32_t* rows,
                    int64_t n, int64_t F, float* out, int64_t ld_out,
                    kgx_stream_t stream);
/* out[perm[i]] = in[i] for i < n (int32 perm) — CSR-order -> input-order. */
int kgx_scatter_f32(const float* in, const int32_t* perm, int64_t n, float* out,
                    kgx_stream_t stream);

/* ---------------------------------------------------------------------------
 * Synthetic R-MAT edge generator (bench/test input; the reference has no
 * generator — its perf tests use numpy.random, tests/performance/
 * test_large_graphs.py:86-110).  Counter-based and bit-reproducible: edge k of
 * (seed, scale, a, b, c) is the same on every device and in the numpy
 * restatement (oracle/rmat.py).  Probabilities are 24-bit fixed point
 * (p * 2^24).  Raw ids (mod n_nodes) are relabelled by a keyed Feistel
 * permutation.  Writes edges [e_begin, e_begin + e_count).
 * ------------------------------------------------------------------------- */
int kgx_rmat_edges(uint64_t seed, int scale, int64_t n_nodes,
                   uint32_t a24, uint32_t b24, uint32_t c24,
                   int64_t e_begin, int64_t e_count,
                   int32_t* src, int32_t* dst, kgx_stream_t stream);

/* Keep edges whose dst lies in [lo, hi): stream compaction used to carve one
 * rank's destination-range shard out of a generated batch.  n_out (host)
 * receives the count; out arrays need capacity n.  Syncs once.               */
int kgx_select_dst_range(const int32_t* src, const int32_t* dst, int64_t n,
                         int64_t lo, int64_t hi, int32_t* src_out, int32_t* dst_out,
                         void* workspace, size_t workspace_bytes, int64_t* n_out,
                         kgx_stream_t stream);
int kgx_select_workspace_bytes(int64_t n, size_t* bytes);

#ifdef __cplusplus
}
#endif
#endif /* KGX_H_ */
