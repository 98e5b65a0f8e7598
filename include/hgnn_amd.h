/*
 * hgnn_amd.h -- C ABI of the MI355X (gfx950) message-passing hot path.
 *
 * Drop-in boundary: these entry points are what the reference's nn.Module
 * forward()/backward() calls become.  The reference is pure Python/PyTorch
 * (SURVEY.md §0.1), so the Python layer in hgnn-2_amd/ (same import paths as
 * the reference: models.gnns.model_mnb, models.layers.*, functions.*) binds
 * this ABI through ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - every pointer named d_* is device memory (HBM) owned by the caller;
 *  - fp32 tensors are dense, contiguous, in the reference's layouts:
 *      X  (bs, f, Nmax)        node features, channel-major (functions/batching.py:116, 172-174)
 *      XL (bs, 1, Emax)        line-graph input = diag(WL[:, :, 1]) (functions/batching.py:119, 171)
 *      W  (bs, Nmax, Nmax, J+2)  graph operators (functions/operators.py:19-29)
 *      WL (bs, Emax, Emax, J+2)  line-graph operators (functions/operators.py:39-81)
 *      Pm, Pd (bs, Nmax, Emax)   incidence operators (functions/operators.py:43-66)
 *      mask (bs, Nmax, Nmax), mask_lg (bs, Emax, Emax)  (functions/batching.py:113-114, 182-183)
 *      N_batch, E_batch (bs,) int64  (functions/batching.py:99-103)
 *  - outputs are caller-allocated; scratch comes from a caller-allocated
 *    workspace whose size is queried first (no allocation inside any call, so
 *    every call can be captured into a hipGraph);
 *  - `stream` is a hipStream_t passed as void*; every call only enqueues work;
 *  - return value: 0 = HGNN_OK, otherwise an HGNN_ERR_* code (the Python layer
 *    raises RuntimeError, the reference's error behaviour);
 *  - device-side input validation (operator entries outside a graph's real
 *    block, mask/N_batch disagreement) ORs HGNN_DEVERR_* bits into a uint32
 *    word inside the workspace; hgnn_*_error_word() gives its device address.
 *  - no global mutable state: calls are re-entrant, one stream per call.
 *
 * Size limits (a call outside them returns HGNN_ERR_UNSUPPORTED or HGNN_ERR_ARG before anything
 * is enqueued, or -- for data-dependent bounds -- sets a device error bit; the reference has no
 * such limits, the Python layer raises RuntimeError):
 *  - networks: J + 2 in [3, 7] (J <= 5; operator values exact below 2^24 as in the reference's fp32 powers); any d with 2d <= 512 (odd 2d runs the same MFMA GEMMs over a
 *    row stride padded to 4); the GEMMs address each operand through a 32-bit buffer resource,
 *    so every per-call operand must stay under 2 GB -- about 12 K QM9-shape graphs per call at
 *    d = 64 (the 640-wide edge aggregate is the largest; split larger batches); the dense
 *    operator gradient (need_dw) keeps a graph's rows in LDS: Nmax <= ~1200 at J + 2 = 3;
 *  - CCN: receptive-field degree <= 1024 (CCN-1D) / 256 (CCN-2D), f_in and hidden <= 16
 *    (HGNN_DEVERR_CCN_DEGREE for the degree, an error status for the channel counts).
 */
#ifndef HGNN_AMD_H
#define HGNN_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HGNN_ABI_VERSION 1

#define HGNN_OK 0
#define HGNN_ERR_ARG 1          /* invalid argument: null pointer, bad size   */
#define HGNN_ERR_UNSUPPORTED 2  /* configuration not compiled (e.g. J > 3)    */
#define HGNN_ERR_HIP 3          /* HIP launch / runtime failure               */
#define HGNN_ERR_INDEX 4        /* input the reference rejects with IndexError */

#define HGNN_DEVERR_PAD_NONZERO 0x1u  /* operator entry outside the real block */
#define HGNN_DEVERR_MASK 0x2u         /* mask[:, :, 0] != (n < N_batch[b])      */
#define HGNN_DEVERR_SIZES 0x4u        /* N_batch > Nmax, E_batch > Emax, < 0   */
#define HGNN_DEVERR_CCN_SELFLOOP 0x8u /* CCN adjacency lacks a self loop        */
#define HGNN_DEVERR_CCN_DEGREE 0x10u  /* CCN degree above the compiled bound    */
#define HGNN_DEVERR_CCN_ASYM 0x20u    /* CCN adjacency pattern not symmetric    */
#define HGNN_DEVERR_DIAG_ID 0x40u     /* operator slice 0 / 1 (I, D) not diagonal */

int hgnn_abi_version(void);
const char* hgnn_status_string(int status);

/* ------------------------------------------------------------------------
 * Network executor: GNN_lg.forward / GNN_simple.forward + autograd backward.
 *
 * Replaces models/gnns/model_mnb.py:58-66 (GNN_simple.forward) and
 * models/gnns/model_mnb.py:124-129 (GNN_lg.forward) with every layer
 * (models/layers/layers_mnb.py:52-69, 88-95, 189-225, 256-290, 322-358,
 * 379-388), BN (models/layers/batch_normalization.py:34-108) and the
 * aggregation ops graph_oper / P_multi (layers_mnb.py:391-434) fused into one
 * enqueue; hgnn_net_backward is the autograd backward of the same graph
 * (scripts/train_mnb.py:90).
 * ---------------------------------------------------------------------- */
typedef struct hgnn_net_config {
    int32_t kind;      /* 0 = GNN_simple, 1 = GNN_lg                              */
    int32_t order;     /* GNN_lg update order 1, 2, 3 (model_mnb.py:102-119)      */
    int32_t bs;        /* graphs in the batch                                     */
    int32_t nmax;      /* padded node count Nmax (X.shape[2])                     */
    int32_t emax;      /* padded edge-slot count Emax (XL.shape[2]); 0 for simple */
    int32_t f_in;      /* dim_input (X.shape[1])                                  */
    int32_t d;         /* n_features                                              */
    int32_t n_layers;  /* >= 2: layer0, n_layers-2 middle layers, layerlast       */
    int32_t j_tot;     /* J + 2 operator slices (W.shape[3])                      */
    int32_t dim_out;   /* dim_output                                              */
    int32_t training;  /* 1: batch BN statistics + running-stat update; 0: eval   */
    int32_t need_dx;   /* backward: write dX (bs, f_in, nmax)                     */
    int32_t need_dw;   /* backward: write dense dW (bs, nmax, nmax, j_tot)        */
    int32_t reserved;
} hgnn_net_config;

typedef struct hgnn_net_inputs {
    const float* d_X;
    const float* d_XL;       /* NULL for GNN_simple */
    const float* d_W;
    const float* d_WL;       /* NULL for GNN_simple */
    const float* d_Pm;       /* NULL for GNN_simple */
    const float* d_Pd;       /* NULL for GNN_simple */
    const int64_t* d_N_batch;
    const int64_t* d_E_batch; /* NULL for GNN_simple */
    const float* d_mask;
    const float* d_mask_lg;   /* NULL for GNN_simple */
} hgnn_net_inputs;

/* Parameter pointer order (device fp32, contiguous), per layer l = 0..n_layers-2:
 *   GNN_lg:     cv1.w cv1.b cv2.w cv2.b bn1.w bn1.b cv3.w cv3.b cv4.w cv4.b bn2.w bn2.b
 *   GNN_simple: cv1.w cv1.b cv2.w cv2.b bn1.w bn1.b
 * then layerlast.fc.w layerlast.fc.b.  BN weight/bias are 0-dim (scalar) tensors
 * (batch_normalization.py:26-27).  Count: hgnn_net_param_count(). */
int hgnn_net_param_count(const hgnn_net_config* cfg);

/* Running BN statistics, per BN module in the order above (bn1, bn2 per layer):
 * running_mean then running_std, each (2 d,).  Updated in place in training
 * mode as r = 0.9 * batch + 0.1 * r (batch_normalization.py:37-38); read in
 * eval mode (batch_normalization.py:41). */
int hgnn_net_bn_count(const hgnn_net_config* cfg);

size_t hgnn_net_workspace_bytes(const hgnn_net_config* cfg);

/* Device address of the validation word inside `workspace` (uint32). */
uint32_t* hgnn_net_error_word(const hgnn_net_config* cfg, void* workspace);

/* out: (bs, dim_out).  The workspace keeps what backward needs; it must stay
 * untouched between a forward and its backward. */
int hgnn_net_forward(const hgnn_net_config* cfg, const hgnn_net_inputs* in,
                     const float* const* params, float* const* bn_running,
                     void* workspace, float* d_out, void* stream);

/* d_dout: (bs, dim_out).  grads: same order/shapes as params; every gradient
 * buffer is OVERWRITTEN.  d_dX (bs, f_in, nmax) if cfg->need_dx, d_dW
 * (bs, nmax, nmax, j_tot) if cfg->need_dw (else may be NULL). */
int hgnn_net_backward(const hgnn_net_config* cfg, const hgnn_net_inputs* in,
                      const float* const* params, void* workspace,
                      const float* d_dout, float* const* grads,
                      float* d_dX, float* d_dW, void* stream);

struct hgnn_csr_batch;  /* defined below (native sparse batcher) */

/* Extended backward: the batch comes from `in` (dense) or `csr` (exactly one non-NULL), an
 * optional launch timer, and optional per-layer completion events for overlapping a gradient
 * all-reduce with the rest of the backward: events[2 l] is recorded on `stream`
 * and events[2 l + 1] on the executor's side stream once every gradient of layer l
 * (l = 0 .. n_layers - 2; layerlast.fc counts as layer n_layers - 2) has been enqueued on
 * that stream -- a communication stream that waits on both may reduce layer l's gradients
 * while layers < l are still being differentiated.  events: hipEvent_t handles;
 * n_events = 2 (n_layers - 1), or 0 for none. */
int hgnn_net_backward_ex(const hgnn_net_config* cfg, const hgnn_net_inputs* in,
                         const struct hgnn_csr_batch* csr, const float* const* params,
                         void* workspace, const float* d_dout, float* const* grads,
                         float* d_dX, float* d_dW, void* stream, void* timer,
                         void* const* events, int n_events);

/* Kernel classes for the optional launch timer (bench.py measures the
 * dominant kernel class and the aggregation classes inside timed regions of
 * its own steps).  A timer times every launch of a class in `class_mask`
 * (bit k = class k) in one of three modes (hgnn_timer_create_ex):
 *   HGNN_TIMER_STAMPS    the aggregation and GEMM kernels write a 100 MHz
 *                        s_memrealtime stamp per wave at entry and exit into
 *                        the timer's device buffer (2 words per wave, stamp_words
 *                        in all); a launch lasts max(exit) - min(entry).  Nothing
 *                        is added to the stream, so a timed kernel runs as in an
 *                        untimed step; classes without stamp slots are not timed;
 *   HGNN_TIMER_DISPATCH  an event pair bound to each dispatch (hipExtLaunchKernel):
 *                        every class, but the timed dispatch runs slower;
 *   HGNN_TIMER_MARKERS   event records on the stream around each launch call.
 * hgnn_timer_create: DISPATCH (MARKERS with HGNN_TIMER_MARKERS=1). */
#define HGNN_TIMER_STAMPS 0
#define HGNN_TIMER_DISPATCH 1
#define HGNN_TIMER_MARKERS 2
#define HGNN_K_STRUCT 0    /* plan, dense->list extraction, pack/unpack */
#define HGNN_K_AGG_FWD 1   /* aggregation gather (graph_oper + P_multi)  */
#define HGNN_K_GEMM_FWD 2  /* fused Conv1d pair GEMM + bias/ReLU/BN partials */
#define HGNN_K_BN_FWD 3    /* BN finalize + apply                         */
#define HGNN_K_READOUT 4   /* readout forward/backward                    */
#define HGNN_K_BN_BWD 5
#define HGNN_K_GEMM_DW 6
#define HGNN_K_GEMM_DA 7
#define HGNN_K_AGG_BWD 8
#define HGNN_K_DW_DENSE 9  /* dense operator gradient dW (W.requires_grad) */
#define HGNN_K_DW_REDUCE 10 /* dW slab + bias reductions                    */
void* hgnn_timer_create(int max_launches, unsigned class_mask);
void* hgnn_timer_create_ex(int max_launches, unsigned class_mask, int mode, long long stamp_words);
void hgnn_timer_reset(void* timer);
/* Waits for the timed work (stamp mode: a device synchronisation and one copy of
 * the stamp buffer); sums the durations of class `kernel_class`. */
int hgnn_timer_elapsed(void* timer, int kernel_class, double* total_ms, int* launches);
/* Stamp mode: every timed launch in enqueue order -- its class, its first-entry / last-exit times in us
 * from the region's earliest stamp (-1: no stamp) and (stream_idx, optional) the stream it went to, numbered
 * in order of first appearance.  Returns the number of launches (up to `max` written), or minus an
 * HGNN_ERR_* code. */
int hgnn_timer_launches(void* timer, int max, int* cls, double* t_entry_us, double* t_exit_us, int* stream_idx);
/* Stamp mode: the entry / exit times (us from the region's earliest stamp, -1: none) of every wave of timed
 * launch `launch` (enqueue order), in the kernel's wave order (linear block id x waves per block + wave).
 * Returns the launch's wave count (up to `max` written), or minus an HGNN_ERR_* code.  (Diagnostics:
 * tools/wave_stats.py.) */
long long hgnn_timer_waves(void* timer, int launch, long long max, double* entry_us, double* exit_us);
void hgnn_timer_destroy(void* timer);
int hgnn_net_forward_timed(const hgnn_net_config* cfg, const hgnn_net_inputs* in,
                           const float* const* params, float* const* bn_running,
                           void* workspace, float* d_out, void* stream, void* timer);
int hgnn_net_backward_timed(const hgnn_net_config* cfg, const hgnn_net_inputs* in,
                            const float* const* params, void* workspace,
                            const float* d_dout, float* const* grads,
                            float* d_dX, float* d_dW, void* stream, void* timer);

/* ------------------------------------------------------------------------
 * Native operator builder and sparse batcher (host C++, csrc/builder.cpp).
 *
 * hgnn_graph_operators replaces graph_operators (functions/operators.py:11-83,
 * twin preprocessing/preprocessing.py:100-170): dense per-graph W (n, n, J+2) and,
 * with dual, WL (m, m, J+2), Pm, Pd (n, m), m = hgnn_graph_edge_slots(n, A) =
 * nnz(A) incl. the diagonal.  Bit-exact, edge-slot quirk included.  Returns
 * HGNN_ERR_INDEX where the reference raises IndexError.
 *
 * hgnn_csr_batch_plan / _build replace prepare_batch (functions/batching.py:77-185)
 * for the executor: a batch of graphs (A_b (n_b, n_b), X_b (n_b, f_in) row-major,
 * host memory) goes straight into one host image holding the packed operator row
 * lists the executor walks, packed X / XL and the batch offsets.  Plan gives the
 * layout (byte offsets, sizes); build fills an image of layout.bytes bytes; the
 * caller copies it to the device and describes it with hgnn_csr_batch_view.
 * ---------------------------------------------------------------------- */
typedef struct hgnn_csr_layout {
    int32_t bs, nmax, emax, f_in, j_tot, dual, stride_w, reserved;
    int64_t nodes, edges;      /* packed node rows, packed edge-slot rows          */
    int64_t rows[6], nnz[6];   /* per list kind: W, WT, WL, WLT, PN (node->slot), PE */
    int64_t off_node_off, off_edge_off, off_totals, off_n_batch, off_e_batch, off_x, off_xl;
    int64_t off_rows[6], off_entries[6];
    int64_t bytes;
} hgnn_csr_layout;
int hgnn_graph_edge_slots(int n, const float* A);
int hgnn_graph_operators(int n, const float* A, int J, int dual, float* W, int m, float* WL,
                         float* Pm, float* Pd);
int hgnn_csr_batch_plan(int bs, const int* n_nodes, const float* const* A, int f_in, int J, int dual,
                        hgnn_csr_layout* layout);
int hgnn_csr_batch_build(int bs, const int* n_nodes, const float* const* A, const float* const* X,
                         int f_in, int J, int dual, const hgnn_csr_layout* layout, void* image);

/* Device view of a CSR batch image (d_base = its device copy). */
typedef struct hgnn_csr_batch {
    const void* d_node_off;    /* int32 (bs + 1) */
    const void* d_edge_off;    /* int32 (bs + 1) */
    const void* d_totals;      /* int32 [nodes, edges] */
    const int64_t* d_n_batch;  /* (bs,) */
    const int64_t* d_e_batch;
    const float* d_x;          /* packed [nodes][f_in] */
    const float* d_xl;         /* packed [edges] */
    const void* d_rows[6];
    const float* d_entries[6];
    int32_t stride_w, reserved;
    int64_t nodes, edges;
} hgnn_csr_batch;
int hgnn_csr_batch_view(const hgnn_csr_layout* layout, const void* d_base, hgnn_csr_batch* out);

/* The executor on a CSR batch: cfg->bs / nmax / emax / f_in / j_tot from the
 * layout; no dense operator, mask or padding is read (no plan / extraction
 * pass).  Backward: need_dw must be 0 (there is no dense W); d_dX is packed
 * [nodes][f_in]. */
int hgnn_net_forward_csr(const hgnn_net_config* cfg, const hgnn_csr_batch* batch,
                         const float* const* params, float* const* bn_running,
                         void* workspace, float* d_out, void* stream);
int hgnn_net_backward_csr(const hgnn_net_config* cfg, const hgnn_csr_batch* batch,
                          const float* const* params, void* workspace,
                          const float* d_dout, float* const* grads, float* d_dX, void* stream);

/* ------------------------------------------------------------------------
 * Device-resident training step (csrc/train.hip): the loss and optimizer of
 * train_with_mnb (scripts/train_mnb.py:41-91) with no host round trip.
 *
 * hgnn_mse_loss: T' = normalize_data(T, mean, std) (functions/utils.py:84-95:
 * mean only when std < 1e-5), d_stats[0] = MSELoss(out, T'), d_stats[1] = MAE
 * (utils.evaluation, functions/utils.py:98-102), d_stats[2..3] = RunningAverage
 * (momentum 0.1, functions/utils.py:134-146) of both, updated in place (zero them
 * per epoch); d_dout (optional) = dLoss/dout = 2 (out - T') / n.
 * hgnn_adamax_step: torch.optim.Adamax(lr, (beta1, beta2), eps, weight_decay)
 * (scripts/main_gnn_qm9.py:185) on n_tensors parameter tensors in one launch per
 * 64 tensors; step = the 1-based step count of this update.
 * ---------------------------------------------------------------------- */
int hgnn_mse_loss(const float* d_out, const float* d_t, int n, float t_mean, float t_std, float* d_stats,
                  float* d_dout, void* stream);

/* Classification branch (scripts/train_mnb.py:50-51, nn.CrossEntropyLoss of
 * scripts/main_generate.py:147): d_out (n, c) logits, d_t (n,) class indices stored
 * as float (prepare_batch's T); stats[0] = mean cross entropy, stats[2] its
 * RunningAverage (stats[1], stats[3] untouched: no MAE for classes); d_dout =
 * (softmax - onehot) / n.  A target outside [0, c) or not integral sets *d_err. */
int hgnn_xent_loss(const float* d_out, const float* d_t, int n, int c, float* d_stats,
                   float* d_dout, uint32_t* d_err, void* stream);
int hgnn_adamax_step(int n_tensors, float* const* params, const float* const* grads, float* const* exp_avg,
                     float* const* exp_inf, const int64_t* numel, double lr, double beta1, double beta2,
                     double eps, double weight_decay, long long step, void* stream);

/* ------------------------------------------------------------------------
 * Covariant compositional networks: CCN_1D / CCN_2D forward + backward.
 *
 * Replaces models/compnets/model_ccn.py:41-64 (CCN_1D.forward) and 93-105
 * (CCN_2D.forward) with CompnetUtils' receptive fields / chi matrices
 * (functions/utils_ccn.py:66-222), promotions and updates (225-324) and
 * collapse6to3 (functions/contraction.py:106-121, evaluated in its O(n^3) closed
 * form).  A batch of graphs is padded like prepare_batch does for the GNNs:
 *   X (bs, nmax, f), adj (bs, nmax, nmax) WITH self loops (scripts/train_ccn.py:36),
 *   n_batch (bs,) int64.
 * Graphs are independent: output[b] is the reference's net(X_b, adj_b).
 * Params: w1.weight w1.bias ... wL.weight wL.bias fc.weight fc.bias (nn.Linear).
 * ---------------------------------------------------------------------- */
typedef struct hgnn_ccn_config {
    int32_t order;    /* 1: CCN_1D, 2: CCN_2D                         */
    int32_t bs, nmax, f_in;
    int32_t hidden;   /* hidden_size                                   */
    int32_t layers;   /* number of update layers (<= 15)               */
    int32_t n_out;    /* n_outputs                                     */
    int32_t reserved;
} hgnn_ccn_config;

/* Plan: receptive fields, degrees, offsets and chi position maps (device).  The
 * one synchronising call of the CCN path: it returns h_sums[4] = {sum d_i,
 * sum d_i^2, nodes, max d_i} to size the feature workspace and the kernels' LDS.
 * Pass the bound max_sum_d2 used to size plan_ws (e.g. bs * nmax^2); HGNN_ERR_ARG
 * if exceeded.  forward / backward / workspace_bytes take the same four sums. */
size_t hgnn_ccn_plan_bytes(const hgnn_ccn_config* cfg, long long max_sum_d2);
int hgnn_ccn_plan(const hgnn_ccn_config* cfg, const float* d_adj, const int64_t* d_n_batch,
                  void* plan_ws, long long max_sum_d2, long long* h_sums, void* stream);
/* Same without any host synchronisation (the per-graph drop-in path, scripts/train_ccn.py:52):
 * h_sums_bound[4] receives upper bounds {bs nmax^2, max_sum_d2, bs nmax, nmax} that size the workspace;
 * the kernels read the exact totals on the device.  max_sum_d2 >= bs nmax^3 (a bound for any
 * content; HGNN_ERR_ARG otherwise), so the sizes never depend on the data. */
int hgnn_ccn_plan_async(const hgnn_ccn_config* cfg, const float* d_adj, const int64_t* d_n_batch,
                        void* plan_ws, long long max_sum_d2, long long* h_sums_bound, void* stream);
uint32_t* hgnn_ccn_error_word(const hgnn_ccn_config* cfg, void* plan_ws, long long max_sum_d2);
size_t hgnn_ccn_workspace_bytes(const hgnn_ccn_config* cfg, const long long* sums);
int hgnn_ccn_forward(const hgnn_ccn_config* cfg, const long long* sums, const float* d_X,
                     const float* const* params, void* plan_ws, long long max_sum_d2,
                     void* workspace, float* d_out, void* stream);
/* grads overwritten (params order); d_dX (bs, nmax, f) overwritten. */
int hgnn_ccn_backward(const hgnn_ccn_config* cfg, const long long* sums, const float* const* params,
                      void* plan_ws, long long max_sum_d2, void* workspace, const float* d_dout,
                      float* const* grads, float* d_dX, void* stream);

/* CCN on small graphs -- order 1 (CCN_1D): nmax <= 64, f_in and hidden <= 8; order 2 (CCN_2D):
 * nmax <= 32, f_in <= 8, hidden <= 2 (the reference's CCN_2D hidden size).  One workgroup per graph
 * builds the receptive fields, runs every level and the readout -- no plan, no host sync, one
 * dispatch forward, one backward (+ one reduction over the graphs when bs > 1).  The per-graph
 * drop-in call of scripts/train_ccn.py:31-73 (net(X, A + I) per graph) and QM9-size batches.  Same
 * layouts and results as hgnn_ccn_forward / _backward: outputs and dX in the same fp32 order (order 2
 * at bs = 1: the weight gradients too -- a batch of several graphs reduces its per-node parameter
 * partials in another order; order 1 sums them in a different order).  d_n_batch may be NULL (every
 * graph has nmax nodes).
 * supported: 1 if cfg fits (order 1: the LDS of the backward, 4 nmax^2 (hidden L + 2 max(f_in, hidden)
 * + 2 hidden) + 8 KB, within 160 KB; order 2: 8 waves x (6.5 KB + 10 nmax^2 B) + 8 KB), else 0 (use
 * the general path).  Order 2's workspace holds each graph's levels at a bound of nmax^3 rows per
 * level: (L + 2) nmax^3 hidden floats per graph (about 4 MB per graph at nmax = 32, L = 15) -- the
 * Python layer sends batches above 512 MB of that region to the general path (hgnn_amd/ccn.py).
 * Validation (self loops, symmetric pattern, 0 <= n_b <= nmax): a graph with bits stores
 * *d_err = tag * 256 + bits (0 < tag < 2^23, a plain store; nothing is stored when the batch is valid;
 * tag only labels the store).  The caller reports any nonzero word and clears it (clear-on-report): a
 * store that lands between the caller's read and its clear is lost.  d_err may be the device alias of
 * a host-mapped word (hgnn_host_word_alloc): the check is then a host read, with no copy or event per
 * call.
 * The workspace holds the readout features between forward and backward. */
int hgnn_ccn_small_supported(const hgnn_ccn_config* cfg);
/* A 64-byte host-mapped, coherent word block (zeroed): *host_ptr for the host, *dev_ptr for kernels. */
int hgnn_host_word_alloc(void** host_ptr, void** dev_ptr);
size_t hgnn_ccn_small_workspace_bytes(const hgnn_ccn_config* cfg);
int hgnn_ccn_small_forward(const hgnn_ccn_config* cfg, const float* d_X, const float* d_adj,
                           const int64_t* d_n_batch, const float* const* params, void* workspace,
                           int32_t* d_err, int32_t tag, float* d_out, void* stream);
int hgnn_ccn_small_backward(const hgnn_ccn_config* cfg, const float* d_X, const float* d_adj,
                            const int64_t* d_n_batch, const float* const* params, void* workspace,
                            const float* d_dout, float* const* grads, float* d_dX, void* stream);

/* collapse6to3 (functions/contraction.py:106-121) on a general 6-D tensor
 * F (C, n, n, n, n, n) -> (n, n, 18 C); the 18 contractions of _c6to2_111 /
 * _c6to2_12 / _c6to2_3 with their diagonal filters. */
int hgnn_collapse6to3(const float* d_F, float* d_out, int c, int n, void* stream);
int hgnn_collapse6to3_backward(const float* d_dout, float* d_dF, int c, int n, void* stream);

/* Byte offsets inside plan_ws of: node_off, deg, nbr (nmax slots per node),
 * selfpos, graph, off1 (prefix of d), off2 (prefix of d^2), pos (chi position
 * maps), error word -- for inspection / tests of the index construction. */
int hgnn_ccn_plan_offsets(const hgnn_ccn_config* cfg, long long max_sum_d2, size_t* offs);

/* ------------------------------------------------------------------------
 * Layer-level drop-ins on dense padded tensors.
 * ---------------------------------------------------------------------- */

/* graph_oper.forward (models/layers/layers_mnb.py:395-411) == graph_op
 * (functions/utils.py:24-52):  out[b, j*F+f, n] = sum_m A[b,n,m,j] X[b,f,m].
 * A (bs, N, N, J), X (bs, F, N), out (bs, J*F, N). */
int hgnn_graph_oper_forward(const float* d_A, const float* d_X, float* d_out,
                            int bs, int n, int j, int f, void* stream);
/* Backward: dX (bs, F, N) = sum_j A_j^T dOut_j (overwritten); dA (bs, N, N, J)
 * = dOut_j X^T if d_dA != NULL (overwritten). */
int hgnn_graph_oper_backward(const float* d_A, const float* d_X, const float* d_dout,
                             float* d_dX, float* d_dA, int bs, int n, int j, int f,
                             void* stream);

/* P_multi.forward (layers_mnb.py:418-434) == Pmul (functions/utils.py:55-81):
 * out[b, f, n] = sum_m P[b, n, m] X[b, f, m], P read as (bs, N, M) with strides
 * (sb, sn, sm) so a transposed view (Pm.transpose(2,1)) needs no copy. */
int hgnn_p_multi_forward(const float* d_P, long sb, long sn, long sm,
                         const float* d_X, float* d_out, int bs, int n, int m, int f,
                         void* stream);
int hgnn_p_multi_backward(const float* d_P, long sb, long sn, long sm,
                          const float* d_X, const float* d_dout, float* d_dX,
                          float* d_dP, int bs, int n, int m, int f, void* stream);

/* BN.forward (batch_normalization.py:34-43) with sb_normalization /
 * mean_with_padding / mask_embedding (65-108).  X, out (bs, C, N); mask (bs, N, N);
 * training: writes batch mean/std (C,) to d_mean/d_std; eval: reads them.
 * w, b: 0-dim device scalars. */
int hgnn_bn_forward(const float* d_X, const int64_t* d_nb, const float* d_mask,
                    const float* d_w, const float* d_b, float* d_mean, float* d_std,
                    float* d_out, int bs, int c, int n, int training, void* stream);
/* dX (bs, C, N) overwritten; dw, db (scalars) overwritten; d_scratch: 2 C floats. */
int hgnn_bn_backward(const float* d_X, const int64_t* d_nb, const float* d_mask,
                     const float* d_w, const float* d_mean, const float* d_std,
                     const float* d_dout, float* d_dX, float* d_dw, float* d_db,
                     float* d_scratch, int bs, int c, int n, int training, void* stream);

/* 1x1 Conv1d (torch.nn.Conv1d(cin, cout, 1), used by every layer_* module,
 * layers_mnb.py:36-37, 81, 172-177, 239-244, 305-310, 371) on the channel-major
 * layout: y (bs, cout, n) = W (cout, cin) . x (bs, cin, n) + b, then ReLU if relu.
 * Workspace: hgnn_conv1x1_workspace_bytes(). */
size_t hgnn_conv1x1_workspace_bytes(int bs, int cin, int cout, int n);
int hgnn_conv1x1_forward(const float* d_x, const float* d_w, const float* d_b, float* d_y,
                         int bs, int cin, int cout, int n, int relu, void* workspace, void* stream);
/* d_dy: gradient wrt the pre-ReLU output.  dW (cout, cin), db (cout) overwritten;
 * dx (bs, cin, n) overwritten when non-NULL. */
int hgnn_conv1x1_backward(const float* d_x, const float* d_w, const float* d_dy, float* d_dx,
                          float* d_dw, float* d_db, int bs, int cin, int cout, int n,
                          void* workspace, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* HGNN_AMD_H */
