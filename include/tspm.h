/*
 * tspm.h — C ABI of the MI355X-native AVMNIST late-fusion training path (libtspm.so, gfx950).
 *
 * Drop-in boundary for the reference's hot path (TArsenii/task-specific-pretraining-multimodal,
 * MML_Suite; paths below are relative to MML_Suite/).  The reference is pure Python/PyTorch: each
 * entry point here replaces the ATen op family that the cited reference line dispatches.  The
 * Python host side (task-specific-pretraining-multimodal_amd/_lib.py) binds these with ctypes —
 * the stub a maintainer adds to the reference is shown in INTEGRATION.md.
 *
 * Conventions
 *   - Every pointer is a DEVICE pointer unless stated otherwise; sizes are element counts.
 *   - Activations are "HWNC": rows ordered (h, w, n), C contiguous fp32 per row.
 *   - Conv weights are OHWI fp32 (the channels_last view of the reference's OIHW nn.Conv2d weight;
 *     the state_dict keeps shape [O, I, H, W]).
 *   - No entry point allocates, synchronises the host, reads the environment or keeps mutable global state
 *     (ABI 21; tspm_flag_create / _destroy below are the one documented allocating pair); workspace is
 *     caller-provided (size queries provided).  Every call is enqueued on `stream` (a hipStream_t),
 *     so calls are capturable into a hipGraph.
 *   - Return value: TSPM_OK (0) or a TSPM_ERR_* code; nothing is launched on error.
 */
#ifndef TSPM_H_
#define TSPM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* tspm_stream_t; /* hipStream_t */

enum {
  TSPM_OK = 0,
  TSPM_ERR_INVALID = 1,   /* bad shape / null pointer / unsupported configuration */
  TSPM_ERR_LAUNCH = 2,    /* the HIP launch failed (hipGetLastError != hipSuccess) */
  TSPM_ERR_WORKSPACE = 3, /* caller-provided workspace too small */
};

/* Version of this ABI (bumped on any signature change; 18 = round 5: the entry points no step calls removed —
 * tspm_conv_fwd_bnin, tspm_conv_wgrad_t, tspm_conv_dgrad_bnfuse / _bwd_bnfuse / _dgrad_bn_tiles,
 * tspm_bn_bwd_apply / _max_tiles, tspm_debug_barrier_timeouts, tspm_bn1d_bwd_maxout — and the 2x2 LDS tiles;
 * 19 = tspm_bn_bwd_src, the BN backward reading its gradient through a pooling layer's backward, and
 * tspm_bn_apply_maxpool, the stem's apply + ReLU + max pool in one launch, and tspm_set_conv_lds_floor (gone in 21);
 * 20 = tspm_conv_bwd_adam, the fused backward launch carrying an Adam update over earlier-finished parameters,
 * and tspm_head_desc.adam_step; 21 = round 6: no mutable global state and no environment reads inside the library —
 * tspm_set_conv_lds_floor removed, the floor and the hand-off mode are per-call tspm_conv_algo fields, and the
 * head's row block is tspm_head_desc.rows_per_block); 22 = round 6: tspm_conv_algo.variant 4, the LDS-staged kernels with
 * every fp32 product formed from an exact three-piece bf16 split on the bf16 MFMA (same structs and entry points). */
#define TSPM_ABI_VERSION 22
int tspm_abi_version(void);  /* returns TSPM_ABI_VERSION */
/* Static string for a status code. */
const char* tspm_status_string(int status);

/* ------------------------------------------------------------------------------------------------
 * Convolution (implicit GEMM on v_mfma_f32_32x32x2_f32, exact fp32)
 * Replaces nn.Conv2d forward / input-grad / weight-grad at models/msa/networks/resnet.py:25,30
 * (3x3 s1/s2 p1), :137 (7x7 s2 p3 stem, Cin=1) and :176 (1x1 s2 downsample); no bias.
 * ----------------------------------------------------------------------------------------------*/
typedef struct tspm_conv_shape {
  int32_t n, h, w, c;  /* input batch, height, width, channels */
  int32_t k, r, s;     /* output channels, kernel height, kernel width */
  int32_t stride, pad; /* symmetric stride / zero padding */
  int32_t p, q;        /* output height, width (= (h + 2 pad - r) / stride + 1, ...) */
} tspm_conv_shape;

/* Tile / split configuration.  tm, tn: 32x32 MFMA tiles per wave along M (rows) and N (columns).
 * variant 0 — register-direct kernels (operands loaded straight into MFMA fragments): a workgroup
 *   holds wn x wk waves: wn neighbouring column tiles of the same rows and wk waves that split the
 *   reduction of one tile and combine through LDS in fixed order (deterministic, no workspace);
 *   splits: additional split of the wgrad reduction over workgroups (fp32 slabs, summed in slab
 *   order).  Supported: (tm,tn) in {(1,1),(1,2),(2,2)}, wn in {1,2,4}, wk in {1,2,4,8,16},
 *   wn*wk <= 8 when wn > 1, wk == 16 only with wn == 1, at most 160 KiB of LDS for the combine.
 *   All-zero fields select the built-in heuristic.
 * variant 1 — LDS-staged kernels (operand stages fetched in full 128-B lines, double-buffered in
 *   LDS): a workgroup is 4 waves = wm x wn x wk with wm = 4 / (wn*wk); tile (wm*tm*32) x (wn*tn*32);
 *   wk waves split every 32-deep reduction stage; splits: split-K over workgroups for fwd, dgrad
 *   and wgrad (fp32 slabs in the workspace, reduced in slab order in-launch).  tm, tn in {1,2}.
 *   Needs HWNC operands, n % (wm*tm*32) == 0 (fwd/dgrad), c % 32 == 0 (fwd), k % 32 == 0 (dgrad),
 *   n % 32 == 0 and c % (wn*tn*32) == 0 (wgrad); otherwise the call returns TSPM_ERR_INVALID.
 *   The workgroup also carries 4 loader waves that stage each operand stage through registers (3 stages
 *   of loads in flight) into two LDS slots.
 * variant 2 — the same tiles and rules with single-role waves: the 4 waves issue the operand loads
 *   themselves as LDS-DMA into a 2-4-slot ring (faster for the batch-256 / 1024 grids; ABI 15).
 * variant 4 — variant 1's kernels (same tiles, splits, epilogues, fused launches) with every fp32 product formed on
 *   the bf16 matrix cores: the loader waves split each fp32 operand exactly into three bf16 pieces (x = h + m + l,
 *   h = x truncated to bf16, m the remainder truncated, l what is left: at most 8 significant bits each, so exact) and
 *   each 16-deep step of a 32x32 tile is the 9 v_mfma_f32_32x32x16_bf16 of the piece pairs — each product x*w is formed
 *   exactly as the sum of its 9 exact parts in the fp32 accumulator; the sign of the staged A operand and of the
 *   accumulator alternates per stage so the bf16 MFMA's truncating accumulation does not bias long reductions.
 *   wk <= 2 (the waves take whole 16-deep steps).  Round 6, ABI 22.
 * variant 3 — the ResNet stems only (c == 1, 7x7, stride 2, pad 3, k == 64; forward and weight
 *   gradient; the other fields are ignored): a workgroup owns one image and a band of output rows,
 *   stages the band's input rows (and, for the weight gradient, its dy rows) in LDS and runs the band
 *   on MFMA.  The forward's BN partial statistics are per band (tspm_conv_fwd_tiles /
 *   _tile_rows report the band count and rows); the weight gradient reduces per-workgroup slabs in
 *   the workspace after its TSPM_COUNTER_BYTES header (tspm_conv_wgrad_workspace).  Round 4.
 * lds_floor (ABI 21; variants 1 and 2): minimum dynamic LDS in bytes (<= 160 KiB; 0 = none) of this launch — a
 *   floor caps how many of the launch's workgroups share a CU, so a concurrent stream keeps CU room (the step sets
 *   it on the encoder with slack).  Scheduling only: results are bitwise the same.  For tspm_conv_bwd[_adam] the
 *   larger of the two algos' floors applies.  (Replaces ABI 19-20's process-wide tspm_set_conv_lds_floor.)
 * flags (ABI 21): TSPM_ALGO_HANDOFF_ACQUIRE — the split-K / BN-merge last arrivers take an agent-scope acquire
 *   before plain loads instead of reading the write-through payload with sc1 loads (bitwise the same; the
 *   reference side of tests/test_gpu_handoff.py, not a performance option). */
#define TSPM_ALGO_HANDOFF_ACQUIRE 1
typedef struct tspm_conv_algo {
  int32_t tm, tn, wn, wk, splits;
  int32_t variant;
  int32_t lds_floor;
  int32_t flags;
} tspm_conv_algo;

/* Element strides (n, h, w, c) of a conv input tensor.  HWNC tensors: {c, w*n*c, n*c, 1}.
 * The reference's NCHW stem input [N,1,H,W] / [N,H,W]: {h*w, w, 1, 0}. */
typedef struct tspm_strides4 {
  int64_t sn, sh, sw, sc;
} tspm_strides4;

/* BatchNorm statistics produced by the convolution epilogue (BatchNorm2d after every conv,
 * resnet.py:25-26,30-31,137-138,176-177).  partial: 3 planes of [tiles][K] floats (tile shift K,
 * mean offset, M2; tiles and rows per tile from the two queries below).  If counters != NULL the
 * last workgroup to finish each column block merges the partials in-launch (no tspm_bn_finalize
 * launch) and writes save_mean / save_invstd and the running statistics: counters = one uint32 per
 * 32 output channels, zero before first use (left zero after every launch).  With counters == NULL
 * only the partials are written (merge them with tspm_bn_finalize).
 * counters_len / partial_floats (ABI 10; 0 = the sizes above): when they reach
 * tspm_conv_fwd_bn_counters / tspm_conv_fwd_bn_partial_floats, a layer with too many tiles for one
 * merging workgroup is merged in two levels inside the launch (groups of tiles by their group's
 * last workgroup into a second partial array after the first, then the groups by the last group)
 * instead of by a tspm_bn_finalize launch. */
typedef struct tspm_bn_fuse {
  float* partial;
  uint32_t* counters;
  float* running_mean; /* nullable */
  float* running_var;  /* nullable */
  float momentum, eps;
  float* save_mean;
  float* save_invstd;
  int32_t counters_len;
  int32_t reserved_;
  int64_t partial_floats;
} tspm_bn_fuse;

/* y[P,Q,N,K] = conv(x, w).  y is HWNC.  bn: NULL, or the BatchNorm statistics to produce from the
 * epilogue (see tspm_bn_fuse) — the conv output is never re-read for them.  Workspace
 * (tspm_conv_fwd_workspace; nonzero only for variant-1 split-K): TSPM_COUNTER_BYTES of arrival
 * counters, zero before first use and left zero, followed by the fp32 slabs. */
int tspm_conv_fwd(const tspm_conv_shape* shape, const tspm_conv_algo* algo, const float* x,
                  const tspm_strides4* x_strides, const float* w, float* y, const tspm_bn_fuse* bn,
                  void* workspace, size_t workspace_bytes, tspm_stream_t stream);
int32_t tspm_conv_fwd_tiles(const tspm_conv_shape* shape, const tspm_conv_algo* algo);
int32_t tspm_conv_fwd_tile_rows(const tspm_conv_shape* shape, const tspm_conv_algo* algo);
/* Buffer sizes that enable the two-level in-launch BN merge (tspm_bn_fuse.counters_len /
 * partial_floats) for this shape and algo. */
int32_t tspm_conv_fwd_bn_counters(const tspm_conv_shape* shape, const tspm_conv_algo* algo);
int64_t tspm_conv_fwd_bn_partial_floats(const tspm_conv_shape* shape, const tspm_conv_algo* algo);
size_t tspm_conv_fwd_workspace(const tspm_conv_shape* shape, const tspm_conv_algo* algo);

/* Round 6 (ABI 21): two independent LDS-staged forwards in ONE launch — the first 3x3 conv of a downsampling
 * BasicBlock and its 1x1 downsample, which read the same block input (resnet.py:41,50-51).  Each half is exactly
 * tspm_conv_fwd with its own shape, algo, operands, BN fuse and workspace (outputs, BN statistics and running stats
 * bitwise those of the two separate calls); the algos must share (tm, tn, wn, wk, variant) — splits and lds_floor
 * may differ (the launch takes the larger floor).  The two BN fuses need distinct partial / counter buffers and two
 * split-K halves distinct workspaces.  TSPM_ERR_INVALID (nothing launched) when the pair is not supported. */
int32_t tspm_conv_fwd_pair_supported(const tspm_conv_shape* s1, const tspm_conv_algo* a1, const tspm_strides4* xs1,
                                     const tspm_conv_shape* s2, const tspm_conv_algo* a2, const tspm_strides4* xs2);
int tspm_conv_fwd_pair(const tspm_conv_shape* s1, const tspm_conv_algo* a1, const float* x1,
                       const tspm_strides4* xs1, const float* w1, float* y1, const tspm_bn_fuse* bn1, void* ws1,
                       size_t ws1_bytes, const tspm_conv_shape* s2, const tspm_conv_algo* a2, const float* x2,
                       const tspm_strides4* xs2, const float* w2, float* y2, const tspm_bn_fuse* bn2, void* ws2,
                       size_t ws2_bytes, tspm_stream_t stream);

/* dx[H,W,N,C] (HWNC) = beta * dx + conv_input_grad(dy[P,Q,N,K], w), beta in {0, 1}.  Workspace
 * (tspm_conv_dgrad_workspace) only for variant-1 split-K, laid out as for the forward. */
int tspm_conv_dgrad(const tspm_conv_shape* shape, const tspm_conv_algo* algo, const float* dy,
                    const float* w, float* dx, int32_t beta, void* workspace, size_t workspace_bytes,
                    tspm_stream_t stream);
size_t tspm_conv_dgrad_workspace(const tspm_conv_shape* shape, const tspm_conv_algo* algo);

/* dw[K,R,S,C] (OHWI) = conv_weight_grad(x, dy[P,Q,N,K]); overwritten (zero_grad semantics).
 * With splits > 1 the workspace holds TSPM_COUNTER_BYTES of arrival counters followed by the fp32
 * slabs; the last workgroup of each tile sums the slabs in slab order in-launch.  The counter
 * header must be zero before the first call (it is left zero after every call), so one zeroed
 * workspace can serve every wgrad shape. */
#define TSPM_COUNTER_BYTES 65536
int tspm_conv_wgrad(const tspm_conv_shape* shape, const tspm_conv_algo* algo, const float* x,
                    const tspm_strides4* x_strides, const float* dy, float* dw, void* workspace,
                    size_t workspace_bytes, tspm_stream_t stream);
size_t tspm_conv_wgrad_workspace(const tspm_conv_shape* shape, const tspm_conv_algo* algo);

/* Input AND weight gradient of one convolution in ONE launch (both algos variant 1): the dgrad and
 * wgrad implicit GEMMs read the same dy and are independent, and at batch 128 either alone leaves
 * most of the 256 CUs idle, so their workgroups share one grid.  Results are bitwise those of
 * tspm_conv_dgrad(algo_dgrad, beta) + tspm_conv_wgrad(algo_wgrad).  Workspaces as for those two
 * calls, one each (not the same buffer when both algos split).  Only the (dgrad, wgrad) tile pairs
 * built into the library run fused: tspm_conv_bwd_supported() returns 1 for those, 0 otherwise
 * (then call the two entry points; tspm_conv_bwd returns TSPM_ERR_INVALID). */
int32_t tspm_conv_bwd_supported(const tspm_conv_shape* shape, const tspm_conv_algo* algo_dgrad,
                                const tspm_conv_algo* algo_wgrad, const tspm_strides4* x_strides);
int tspm_conv_bwd(const tspm_conv_shape* shape, const tspm_conv_algo* algo_dgrad,
                  const tspm_conv_algo* algo_wgrad, const float* x, const tspm_strides4* x_strides,
                  const float* dy, const float* w, float* dx, int32_t beta, float* dw, void* ws_dgrad,
                  size_t ws_dgrad_bytes, void* ws_wgrad, size_t ws_wgrad_bytes, tspm_stream_t stream);
/* ------------------------------------------------------------------------------------------------
 * BatchNorm2d, training mode (batch statistics over N*H*W, biased variance for normalisation,
 * unbiased for running_var, momentum 0.1, eps 1e-5) — resnet.py:26,31,138,177.
 * ----------------------------------------------------------------------------------------------*/
/* Batch statistics of y[M,C] (M = N*H*W rows).  If nslab > 1, y holds nslab partial slabs
 * (slab_stride elements apart) that are summed in slab order and written to y_out (the conv output
 * used downstream); with nslab == 1, y_out may be NULL or == y.  Writes save_mean / save_invstd [C]
 * and updates running_mean / running_var in place (if non-NULL).  Workspace: tspm_bn_stats_workspace. */
int tspm_bn_stats(int64_t m, int32_t c, const float* y, int32_t nslab, int64_t slab_stride,
                  float* y_out, float* running_mean, float* running_var, float momentum, float eps,
                  float* save_mean, float* save_invstd, void* workspace, size_t workspace_bytes,
                  tspm_stream_t stream);
size_t tspm_bn_stats_workspace(int64_t m, int32_t c);

/* Merge per-tile partial statistics (3 planes of [ntiles][c]: tile shift K, mean-K, M2; tile t
 * holds min(rows_per_tile, m - t*rows_per_tile) rows) into save_mean / save_invstd and the running
 * statistics — the tail of tspm_bn_stats, and the consumer of tspm_conv_fwd's partials when no
 * counters are given. */
int tspm_bn_finalize(int64_t m, int32_t c, int32_t ntiles, int64_t rows_per_tile, const float* partial,
                     float* running_mean, float* running_var, float momentum, float eps, float* save_mean,
                     float* save_invstd, tspm_stream_t stream);

/* out = act( gamma*(y-mean)*invstd + beta  [+ residual] ), act = ReLU if relu != 0.
 * res_mode 0: no residual; 1: residual = res (raw tensor, same [M,C]); 2: residual =
 * BN(res; res_mean, res_invstd, res_gamma, res_beta) — the downsample branch (resnet.py:47-52). */
int tspm_bn_apply(int64_t m, int32_t c, const float* y, const float* mean, const float* invstd,
                  const float* gamma, const float* beta, int32_t res_mode, const float* res,
                  const float* res_mean, const float* res_invstd, const float* res_gamma,
                  const float* res_beta, int32_t relu, float* out, float* out_t, int64_t ld_t,
                  tspm_stream_t stream);

/* Eval-mode BN (running statistics) with the same fusion options. */
int tspm_bn_apply_eval(int64_t m, int32_t c, const float* y, const float* running_mean,
                       const float* running_var, float eps, const float* gamma, const float* beta,
                       int32_t res_mode, const float* res, const float* res_rmean, const float* res_rvar,
                       const float* res_gamma, const float* res_beta, int32_t relu, float* out,
                       tspm_stream_t stream);

/* ABI 17: the encoder's last block apply with the adaptive average pool folded in.  Rows are
 * position-major (row = p*n + sample, npos positions): out = tspm_bn_apply's result over the npos*n rows
 * (tspm_bn_apply_eval's when eval != 0: mean / inv are then the running mean / variance and eps applies),
 * and pooled[n][c] = (sum over p of out) / npos — tspm_avgpool_fwd of out — in the same launch. */
int tspm_bn_apply_pool(int32_t npos, int32_t n, int32_t c, const float* y, const float* mean, const float* inv,
                       const float* gamma, const float* beta, int32_t res_mode, const float* res,
                       const float* res_mean, const float* res_inv, const float* res_gamma, const float* res_beta,
                       int32_t relu, int32_t eval, float eps, float* out, float* pooled, tspm_stream_t stream);

/* Round 6 (ABI 21): the training-mode apply (as tspm_bn_apply) with the statistics merge of tspm_bn_finalize folded
 * into its prologue, for convs whose forward cannot merge its partials in-launch (tspm_conv_fwd_bn_inlaunch == 0;
 * the caller then passes a tspm_bn_fuse without counters so the conv only writes the partials): every workgroup
 * merges the `tiles` (<= 256) partial tiles of its 16 channels in double in a fixed order, row block 0 writes
 * save_mean / save_invstd and updates the running statistics (momentum, unbiased variance), and its rows are
 * normalised.  One launch instead of tspm_bn_finalize + tspm_bn_apply.  c % 16 == 0. */
int32_t tspm_conv_fwd_bn_inlaunch(const tspm_conv_shape* shape, const tspm_conv_algo* algo);
int tspm_bn_apply_merge(int64_t m, int32_t c, int32_t tiles, int64_t rows_per_tile, const float* partial,
                        float* running_mean, float* running_var, float momentum, float eps, float* save_mean,
                        float* save_invstd, const float* y, const float* gamma, const float* beta, int32_t res_mode,
                        const float* res, const float* res_mean, const float* res_invstd, const float* res_gamma,
                        const float* res_beta, int32_t relu, float* out, tspm_stream_t stream);

/* ABI 19: the stem's BN apply + ReLU with the following MaxPool2d(3, 2, 1) in the same launch (resnet.py:138-140):
 * pooled [p][q][n][c] and its argmax taps idx exactly as tspm_maxpool_fwd over tspm_bn_apply's output, and that
 * output out [h][w][n][c] (nullable; the BN backward's ReLU mask) — bitwise the two launches.  eval != 0: inv is
 * the running variance and eps applies (tspm_bn_apply_eval's arithmetic).  p = (h-1)/2+1, q = (w-1)/2+1. */
int tspm_bn_apply_maxpool(int32_t n, int32_t h, int32_t w, int32_t c, const float* y, const float* mean,
                          const float* inv, const float* gamma, const float* beta, int32_t eval, float eps, float* out,
                          float* pooled, uint8_t* idx, int32_t p, int32_t q, tspm_stream_t stream);

/* BN backward through  out = relu(BN(y) [+ BN2(y2)])  (y2 / second BN optional, may be NULL):
 *   g' = g * (out > 0)  (out may be NULL: no ReLU)
 *   dgamma = sum(g' * xhat), dbeta = sum(g')          (written, not accumulated)
 *   dy  = gamma*invstd*(g' - dbeta/M - xhat*dgamma/M)
 *   dy2 likewise for the second BN; if dres != NULL it receives g' (identity residual grad).
 * dy_t / dy2_t (nullable): also write dy / dy2 transposed, [c][ld_t] with the m = (h*W + w)*N + n rows of
 * channel c contiguous (ld_t >= m, ld_t % 4 == 0, 16-byte aligned); no step uses them.
 * Workspace: tspm_bn_bwd_workspace bytes (per-tile partial sums); one workspace must not be used by two
 * launches in flight at once. */
int tspm_bn_bwd(int64_t m, int32_t c, const float* g, const float* out, const float* y,
                const float* mean, const float* invstd, const float* gamma, float* dgamma, float* dbeta,
                float* dy, const float* y2, const float* mean2, const float* invstd2,
                const float* gamma2, float* dgamma2, float* dbeta2, float* dy2, float* dres,
                float* dy_t, float* dy2_t, int64_t ld_t, void* workspace, size_t workspace_bytes,
                tspm_stream_t stream);
size_t tspm_bn_bwd_workspace(int64_t m, int32_t c);
/* ABI 19: the same BN backward with its incoming gradient g formed on the fly from a pooling layer's output
 * gradient instead of read from a materialised [m, c] tensor (one launch and the g tensor's write + reads fewer):
 *   kind TSPM_GSRC_AVGPOOL — the encoder's AdaptiveAvgPool2d(1) + flatten (resnet.py:59-60): g[(pos, n)] =
 *     gp[n * ldg + c] / npos, exactly tspm_avgpool_bwd's value (npos = h * w);
 *   kind TSPM_GSRC_MAXPOOL — the stem's MaxPool2d(3, 2, 1) (resnet.py:140): g = tspm_maxpool_bwd's dx from gp
 *     [p][q][n][c] and its argmax taps idx (same window order, bitwise).
 * Rows m = h * w * n (HWNC) < 2^24.  Otherwise as tspm_bn_bwd without the transposed copies. */
enum { TSPM_GSRC_AVGPOOL = 1, TSPM_GSRC_MAXPOOL = 2 };
typedef struct tspm_bn_gsrc {
  int32_t kind;
  int32_t n, h, w;     /* the BN input map: m = h * w * n rows */
  int32_t p, q;        /* maxpool: the pooled map */
  int32_t npos, ldg;   /* avgpool: positions (= h * w) and the row stride of gp [n][ldg] */
  const float* gp;     /* the pooling layer's output gradient */
  const uint8_t* idx;  /* maxpool: argmax taps [p][q][n][c] (tspm_maxpool_fwd) */
} tspm_bn_gsrc;
int tspm_bn_bwd_src(int64_t m, int32_t c, const tspm_bn_gsrc* src, const float* out, const float* y,
                    const float* mean, const float* invstd, const float* gamma, float* dgamma, float* dbeta,
                    float* dy, const float* y2, const float* mean2, const float* invstd2, const float* gamma2,
                    float* dgamma2, float* dbeta2, float* dy2, float* dres, void* workspace, size_t workspace_bytes,
                    tspm_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * Pooling — nn.MaxPool2d(3, 2, 1) (resnet.py:140,208) and AdaptiveAvgPool2d(1)+flatten (:149,215-216)
 * ----------------------------------------------------------------------------------------------*/
/* y[P,Q,N,C] = maxpool(x[H,W,N,C]); argmax tap (0..k*k-1, first max in row-major window order,
 * as ATen's CPU kernel) stored in idx (uint8, same shape as y). */
int tspm_maxpool_fwd(int32_t n, int32_t h, int32_t w, int32_t c, int32_t k, int32_t stride, int32_t pad,
                     int32_t p, int32_t q, const float* x, float* y, uint8_t* idx, float* y_t, int64_t ld_t,
                     tspm_stream_t stream);
/* dx = scatter of dy to the argmax positions (gather form, deterministic); dx overwritten. */
int tspm_maxpool_bwd(int32_t n, int32_t h, int32_t w, int32_t c, int32_t k, int32_t stride, int32_t pad,
                     int32_t p, int32_t q, const float* dy, const uint8_t* idx, float* dx,
                     tspm_stream_t stream);
/* y[N,C] = mean over the npos positions of x[npos,N,C] (HWNC). */
int tspm_avgpool_fwd(int32_t npos, int32_t n, int32_t c, const float* x, float* y, tspm_stream_t stream);
/* dx[npos,N,C] = dy[N,C] / npos (dy row stride ldy). */
int tspm_avgpool_bwd(int32_t npos, int32_t n, int32_t c, const float* dy, int32_t ldy, float* dx,
                     tspm_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * Linear layers — encoder fc (resnet.py:150,217) and the fusion head (models/avmnist.py:219-230,267)
 * w is [out, in] row-major (nn.Linear layout).  ld* are row strides (elements).
 * ----------------------------------------------------------------------------------------------*/
/* y = act(x @ w^T + b) [* keep*scale]; relu != 0 applies ReLU; keep (uint8 [n,out], may be NULL)
 * applies the dropout mask with scale 1/(1-p) (models/avmnist.py:219-230). */
int tspm_linear_fwd(int32_t n, int32_t in, int32_t out, const float* x, int32_t ldx, const float* w,
                    const float* b, int32_t relu, const uint8_t* keep, float keep_scale, float* y,
                    int32_t ldy, tspm_stream_t stream);
/* tspm_linear_fwd with the reduction split over `splits` workgroup slices (ABI 11): for long inputs
 * with few output tiles (the MMIMDb image encoder, 4096 -> 512 at batch 256: 128 tiles for 256 CUs).
 * Partial products go to the workspace (tspm_linear_fwd_splitk_workspace bytes; 0 = no split needed)
 * and a second launch sums the slices in order and applies the epilogue.  Same results as
 * tspm_linear_fwd up to summation order. */
int tspm_linear_fwd_splitk(int32_t n, int32_t in, int32_t out, const float* x, int32_t ldx, const float* w,
                           const float* b, int32_t relu, const uint8_t* keep, float keep_scale, float* y,
                           int32_t ldy, int32_t splits, void* workspace, size_t workspace_bytes,
                           tspm_stream_t stream);
size_t tspm_linear_fwd_splitk_workspace(int32_t n, int32_t in, int32_t out, int32_t splits);
/* Two bias-free Linear forwards of the same shape in one launch (the GMU's fc_one / fc_two,
 * models/gates/gated_bimodal.py; ABI 11): y0 = x0 @ w0^T, y1 = x1 @ w1^T, bitwise tspm_linear_fwd. */
int tspm_linear_fwd_pair(int32_t n, int32_t in, int32_t out, const float* x0, int32_t ldx0, const float* w0,
                         float* y0, int32_t ldy0, const float* x1, int32_t ldx1, const float* w1, float* y1,
                         int32_t ldy1, tspm_stream_t stream);
/* dx = dy @ w  (dx overwritten). */
int tspm_linear_bwd_data(int32_t n, int32_t in, int32_t out, const float* dy, int32_t ldy, const float* w,
                         float* dx, int32_t ldx, tspm_stream_t stream);
/* dw = dy^T @ x, db = sum_n dy (both overwritten). */
int tspm_linear_bwd_weight(int32_t n, int32_t in, int32_t out, const float* x, int32_t ldx,
                           const float* dy, int32_t ldy, float* dw, float* db, tspm_stream_t stream);
/* tspm_linear_bwd_weight with the reduction over the n rows split into `splits` workgroup slices
 * (ABI 13): for very long reductions with few output tiles (the LSTM weight gradients of the MOSI
 * step, n = T*B = 6400 rows into 256 x 64 / 256 x 5 / 256 x 20 outputs).  Per-slice partial products
 * and row sums go to the workspace (tspm_linear_bwd_weight_splitk_workspace bytes; 0 = no split), a
 * second launch sums the slices in order.  Same results as tspm_linear_bwd_weight up to summation
 * order; dw and db from the same call share one split (an LSTM's db_ih / db_hh stay bitwise equal). */
int tspm_linear_bwd_weight_splitk(int32_t n, int32_t in, int32_t out, const float* x, int32_t ldx, const float* dy,
                                  int32_t ldy, float* dw, float* db, int32_t splits, void* workspace,
                                  size_t workspace_bytes, tspm_stream_t stream);
size_t tspm_linear_bwd_weight_splitk_workspace(int32_t n, int32_t in, int32_t out, int32_t splits);
/* Both backward products of one nn.Linear in ONE launch (ABI 11): dw = dy^T @ x, db = sum_n dy
 * (db nullable), and, if dx != NULL, dx = dy @ w (row stride lddx) — bitwise the results of
 * tspm_linear_bwd_weight + tspm_linear_bwd_data (same per-product reduction split). */
int tspm_linear_bwd(int32_t n, int32_t in, int32_t out, const float* x, int32_t ldx, const float* dy, int32_t ldy,
                    const float* w, float* dw, float* db, float* dx, int32_t lddx, tspm_stream_t stream);
/* Backward of up to 2 independent nn.Linear layers in ONE launch (ABI 11; e.g. the GMU's fc_one and
 * fc_two, or the MMIMDb image and text encoder Linears): each descriptor as tspm_linear_bwd (dx
 * nullable), bitwise its results.  descs is a host array read at launch time. */
typedef struct tspm_linear_bwd_desc {
  int32_t n, in, out, ldx, ldy, lddx;
  const float* x;
  const float* dy;
  const float* w;
  float* dw;
  float* db;
  float* dx;
} tspm_linear_bwd_desc;
int tspm_linear_bwd_multi(int32_t count, const tspm_linear_bwd_desc* descs, tspm_stream_t stream);
/* In-place gradient masking through a ReLU(+dropout) output y: g = (y > 0) ? g * scale : 0
 * (scale = 1/(1-p) when y is the post-dropout output — y > 0 implies the unit was kept). */
int tspm_act_bwd(int32_t n, int32_t cols, float* g, int32_t ldg, const float* y, int32_t ldy, float scale,
                 tspm_stream_t stream);

/* Dropout keep mask (uint8) from a counter-based hash RNG: keep[i] = u(seed, ctr, i) >= p, where
 * ctr is read from device memory (*counter) so graph replays draw fresh masks. */
int tspm_dropout_mask(int64_t count, float p, uint64_t seed, const uint64_t* counter, uint8_t* keep,
                      tspm_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * Loss — LossFunctionGroup{cross_entropy: 1.0} (experiment_utils/loss.py:123-148,
 * models/avmnist.py:301) + on-device accuracy counters (avmnist.py:305-309)
 * ----------------------------------------------------------------------------------------------*/
/* loss[0] = grad_scale * mean_i CE(logits_i, labels_i) (the group's total: weight × CE, grad_scale =
 * the term's weight); dlogits = (softmax - onehot)/n * grad_scale;
 * if stats != NULL: stats[0] += loss*n, stats[1] += #correct (argmax == label), stats[2] += n. */
int tspm_cross_entropy(int32_t n, int32_t classes, const float* logits, const int64_t* labels, float* loss,
                       float* dlogits, float grad_scale, float* stats, tspm_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * Fusion head train step (ABI 16) — AVMNIST's classifier `net` = Linear(in, hidden) → ReLU →
 * Dropout(p) → Linear(hidden, hidden2) → ReLU → Linear(hidden2, classes) (models/avmnist.py:219-230,
 * forward :267), the LossFunctionGroup's weighted cross-entropy (experiment_utils/loss.py:98-148) and
 * the head's whole backward, in TWO launches instead of ten:
 *   (1) one sample per workgroup (512 threads; round 5 — rows_per_block = 4 selects round 4's blocks of 4
 *       samples on 256 threads), the three weight matrices staged in LDS: dropout keep
 *       mask (same counter-hash bits as
 *       tspm_dropout_mask, or read from `keep` when gen_keep == 0), h1, hh, logits, per-row CE,
 *       dlogits, dz3 = (dlogits @ w5) * (hh > 0), dz0 = (dz3 @ w3) * (h1 > 0 ? 1/(1-p) : 0) and
 *       dx = dz0 @ w0 (the gradient flowing into the two encoders' embeddings);
 *   (2) the three weight / bias gradients (dw = dz^T @ input, db = column sums; overwritten) on the
 *       small-GEMM tiles, plus one workgroup that reduces the per-row losses in a fixed order:
 *       loss[0] = weight * mean CE, stats[0] += sum CE, stats[1] += #(argmax == label), stats[2] += n.
 * Every buffer below is caller-owned device memory; row_ws holds 2*n floats.  Same semantics as
 * tspm_linear_fwd/_bwd + tspm_act_bwd + tspm_dropout_mask + tspm_cross_entropy (out-of-range label →
 * NaN loss and gradients), up to summation order.  Limits: in <= 256, hidden <= 256, hidden2 <= 128,
 * classes <= 16; in, hidden, hidden2 multiples of 4; w0 / w3 / x rows 16-byte aligned; the three
 * weight matrices plus the row blocks within 160 KiB of LDS (floats, RB = rows per workgroup, logits rows
 * padded to a multiple of 4: hidden*(in+4) + hidden2*(hidden+4) + classes*(hidden2+4)
 * + RB*(in+hidden+hidden2+12+round_up4(classes)) + hidden+hidden2+classes+RB); otherwise TSPM_ERR_INVALID. */
typedef struct tspm_head_desc {
  int32_t n, in, hidden, hidden2, classes, ldx, lddx, gen_keep;
  const float* x;                  /* [n, ldx] the fused embeddings (concat of the two encoders) */
  const float *w0, *b0, *w3, *b3, *w5, *b5;
  float p;                         /* dropout probability (0: no mask) */
  float loss_weight;               /* the cross-entropy term's weight */
  uint64_t seed;
  const uint64_t* counter;         /* device step counter (fresh masks per graph replay) */
  uint8_t* keep;                   /* [n, hidden] */
  const int64_t* labels;           /* [n] */
  float *h1, *hh, *logits, *dlogits, *dz3, *dz0, *dx, *row_ws;
  float *gw0, *gb0, *gw3, *gb3, *gw5, *gb5;
  float *loss, *stats;             /* stats nullable */
  int64_t* adam_step;              /* nullable (ABI 20): the optimizer's tspm_adam_hyper.step, incremented once by
                                    * launch 2 after launch 1 read `counter` (tspm_adam_begin's job, one launch fewer
                                    * between the forward and the backward) */
  int32_t rows_per_block;          /* ABI 21: samples per workgroup of launch 1 — 0 = the default (1 up to 256
                                    * rows, else 4), or 1 / 4 (A/B; was the TSPM_HEAD_RB environment read) */
  int32_t reserved_;
} tspm_head_desc;
int tspm_head_train_step(const tspm_head_desc* desc, tspm_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * Adam — torch.optim.Adam (L2 weight decay folded into the gradient) as instantiated by
 * config/optimizer_config.py:199-226 with lr 5e-4, wd 1e-4 (train_avmnist_resnet.yaml)
 * ----------------------------------------------------------------------------------------------*/
typedef struct tspm_adam_hyper {
  /* doubles, like torch.optim.Adam's Python-float hyper-parameters: 1-beta2 and the bias
   * corrections are formed in double and rounded to fp32 once, as ATen does */
  double lr, beta1, beta2, eps, weight_decay, grad_scale; /* grad_scale multiplies g (e.g. 1/world) */
  int64_t step;                                          /* incremented on device by tspm_adam_begin */
  int64_t pad_;
} tspm_adam_hyper;
/* hyper->step += 1 (device-side, so a captured graph advances the bias correction per replay). */
int tspm_adam_begin(tspm_adam_hyper* hyper, tspm_stream_t stream);
/* counters[i] += value for i < count (ABI 13): every BatchNorm's num_batches_tracked (one shared
 * int64 vector) advanced once per training step inside the captured step. */
int tspm_counters_add(int64_t* counters, int64_t count, int64_t value, tspm_stream_t stream);

/* Step flags (ABI 15) for the DP step's exchange ordering across a graph boundary.  A flag is a device
 * counter plus a word of coherent pinned host memory.  tspm_flag_bump enqueues a one-thread kernel that
 * increments the counter and stores the new value to the host word (system-scope release) — capturable, so
 * it marks a point INSIDE a captured step graph; tspm_flag_host_wait spins on the host until the word is
 * >= value (0 = TSPM_OK; TSPM_ERR_LAUNCH after timeout_ms).  The host then launches work that depends on
 * that point.  (ROCm 7 refuses graph-external event records; a hipStreamWaitValue64 on another stream
 * cost 0.21 ms per step — the waiting queue stalls the graph's.) */
typedef struct tspm_flag tspm_flag;
int tspm_flag_create(tspm_flag** flag);
int tspm_flag_destroy(tspm_flag* flag);
int tspm_flag_bump(tspm_flag* flag, tspm_stream_t stream);
int tspm_flag_host_wait(tspm_flag* flag, uint64_t value, int32_t timeout_ms);
/* One fused Adam update over `count` contiguous fp32 elements (the flat parameter buffer). */
int tspm_adam_step(int64_t count, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                   const tspm_adam_hyper* hyper, tspm_stream_t stream);
/* tspm_adam_step with the gradient also multiplied by the device scalar *clip_coef (ABI 12: the
 * coefficient tspm_grad_clip_coef wrote — torch.nn.utils.clip_grad_norm_ before optimizer.step(),
 * MML_Suite/models/msa/utt_fusion.py:188-190).  g' = (g * grad_scale) * clip_coef. */
int tspm_adam_step_clip(int64_t count, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                        const tspm_adam_hyper* hyper, const float* clip_coef, tspm_stream_t stream);

/* ABI 20: tspm_conv_bwd that also carries an Adam update: `blocks` extra workgroups of the same grid run
 * tspm_adam_step's element loop over `count` elements starting at param / grad / exp_avg / exp_avg_sq (a range of
 * the optimizer's flat buffers whose gradients an EARLIER launch on the stream finished and which no later launch
 * reads), bitwise tspm_adam_step over that range (hyper->step must already be advanced by tspm_adam_begin).  The
 * optimizer pass that follows the backward (MML_Suite train loop: loss.backward(); optimizer.step(),
 * train_multimodal.py) is thereby spread over the backward's latency-bound launches instead of following them.
 * count = 0: plain tspm_conv_bwd. */
typedef struct tspm_adam_job {
  float* param;
  const float* grad;
  float *exp_avg, *exp_avg_sq;
  int64_t count;
  const tspm_adam_hyper* hyper;
  int32_t blocks, pad_;
} tspm_adam_job;
int tspm_conv_bwd_adam(const tspm_conv_shape* s, const tspm_conv_algo* dgrad_algo, const tspm_conv_algo* wgrad_algo,
                       const float* x, const tspm_strides4* x_strides, const float* dy, const float* w, float* dx,
                       int32_t beta, float* dw, const tspm_adam_job* job, void* ws_d, size_t ws_d_bytes, void* ws_w,
                       size_t ws_w_bytes, tspm_stream_t stream);

/* Round 6 (ABI 21): the BatchNorm backward's partial sums formed by the dgrad epilogue that writes its incoming
 * gradient.  In the ResNet backward (resnet.py:37-54 under autograd) the gradient of bn1's output is conv2's input
 * gradient, and the gradient of bn2's output (through the block's ReLU) is the next block's conv1 input gradient
 * accumulated onto the residual branch; the last-arriving workgroup of each dgrad tile holds those values in
 * registers.  With bnp set, tspm_conv_bwd_ex's dgrad epilogue also writes, per 32-row tile t and channel c of dx
 * (after the beta accumulate — dx itself bitwise as without bnp), with g' = dx * [out > 0]:
 *   part[0][t][c] = sum g',  part[1][t][c] = sum g' (y - mean[c]),  part[2][t][c] = sum g' (y2 - mean2[c]) (y2 set)
 * — exactly what tspm_bn_bwd's partial pass computes over its own row tiles, so tspm_bn_bwd_apply_part can run the
 * BN backward's apply (merge + dy) without that pass: one launch fewer per BatchNorm backward.  Needs
 * (h*w*n) % 32 == 0; out, y, y2 are [h*w*n][c] HWNC like dx. */
typedef struct tspm_bn_bwd_part {
  const float* out;    /* the ReLU output that gates the gradient */
  const float* y;      /* the BN's input (its conv output) */
  const float* mean;   /* its save_mean [c] */
  const float* y2;     /* nullable: a second BN fed by the same gradient (the block's downsample branch) */
  const float* mean2;  /* its save_mean [c] */
  float* part;         /* [2 or 3][(h*w*n)/32][c] */
  /* Max-pool gather (nullable idx): dx is the gradient of a MaxPool2d(3, 2, 1) output whose argmax taps are idx
   * ([h][w][n][c] uint8, tspm_bn_apply_maxpool's), and the BN sits before that pool on a pool_h x pool_w map (the
   * ResNet stem, resnet.py:138-140): out / y are read at each pooled element's argmax position, so the sums are the
   * BN backward's over the pool's input-gradient (sum over the map of maxpool_bwd(dx) * [out > 0] ...) formed in
   * the pooled domain — one gathered read per pooled element instead of a pass over the pool's input. */
  const uint8_t* idx;
  int32_t pool_h, pool_w;
  /* Whole BN backward in the same launch (round 6; dy non-null, no idx): the last dgrad tile of each column block
   * to finish (a ticket on counters[column block]: one uint32 per (c / tile columns), zero before first use, left
   * zero) merges that block's partial tiles in tspm_bn_bwd_apply_part's order, writes dgamma / dbeta and applies
   * dy [, dy2] [, dres = g'] over all rows of its channels — tspm_bn_bwd_apply_part's values, no apply launch.
   * dx and the partials are then published write-through (sc1) for it.  Meant for short maps (the tail is one
   * workgroup per column block). */
  const float *invstd, *gamma;
  float *dgamma, *dbeta, *dy;
  const float *invstd2, *gamma2;
  float *dgamma2, *dbeta2, *dy2, *dres;
  uint32_t* counters;
} tspm_bn_bwd_part;
/* tspm_conv_bwd with an optional carried Adam job (as tspm_conv_bwd_adam; nullable) and optional BN-backward
 * partial sums of dx (bnp; nullable). */
int tspm_conv_bwd_ex(const tspm_conv_shape* s, const tspm_conv_algo* dgrad_algo, const tspm_conv_algo* wgrad_algo,
                     const float* x, const tspm_strides4* x_strides, const float* dy, const float* w, float* dx,
                     int32_t beta, float* dw, const tspm_adam_job* job, const tspm_bn_bwd_part* bnp, void* ws_d,
                     size_t ws_d_bytes, void* ws_w, size_t ws_w_bytes, tspm_stream_t stream);
/* Round 6: the backward of a downsampling block's second conv (s, dg, wg: its dgrad + wgrad exactly as
 * tspm_conv_bwd_ex, with the optional bnp) and of the block's 1x1 downsample (s2, dg2, wg2: dgrad with beta 0 into
 * dx2 + wgrad into dw2) in ONE launch — both read gradients the block's bn2 backward has just written and write
 * disjoint tensors (resnet.py:41-51 under autograd).  dg2 / wg2 must have dg / wg's (tm, tn, wn, wk, variant);
 * splits may differ; split-K halves need pairwise distinct workspaces.  job (nullable) as tspm_conv_bwd_adam. */
int32_t tspm_conv_bwd_quad_supported(const tspm_conv_shape* s, const tspm_conv_algo* dg, const tspm_conv_algo* wg,
                                     const tspm_strides4* xs, const tspm_conv_shape* s2, const tspm_conv_algo* dg2,
                                     const tspm_conv_algo* wg2, const tspm_strides4* xs2);
int tspm_conv_bwd_quad(const tspm_conv_shape* s, const tspm_conv_algo* dg, const tspm_conv_algo* wg, const float* x,
                       const tspm_strides4* xs, const float* dy, const float* w, float* dx, int32_t beta, float* dw,
                       const tspm_bn_bwd_part* bnp, void* ws_d, size_t ws_d_bytes, void* ws_w, size_t ws_w_bytes,
                       const tspm_conv_shape* s2, const tspm_conv_algo* dg2, const tspm_conv_algo* wg2,
                       const float* x2, const tspm_strides4* xs2, const float* dy2, const float* w2, float* dx2,
                       float* dw2, void* ws_d2, size_t ws_d2_bytes, void* ws_w2, size_t ws_w2_bytes,
                       const tspm_adam_job* job, tspm_stream_t stream);
/* The BN backward's second launch alone (tspm_bn_bwd's k_bn_bwd_apply_m) over partial sums `part` of `tiles` row
 * tiles ([2 or 3][tiles][c], e.g. from tspm_conv_bwd_ex's bnp; tiles <= 128): every workgroup merges the tiles in
 * double in a fixed order, writes dgamma / dbeta (first row block) and dy = gamma*invstd*(g' - mean(g') -
 * xhat*mean(g' xhat)) [dy2 likewise for y2], dres = g' (nullable).  Arguments otherwise as tspm_bn_bwd with g dense
 * (out required). */
/* tspm_bn_bwd_apply_part with the gradient read through a pooling layer's backward (the stem BN under the max pool:
 * src->kind TSPM_GSRC_MAXPOOL, as tspm_bn_bwd_src), its partial sums from tspm_conv_bwd_ex's max-pool gather mode
 * (tspm_bn_bwd_part.idx); single BN, no dres. */
int tspm_bn_bwd_apply_part_src(int64_t m, int32_t c, int32_t tiles, const float* part, const tspm_bn_gsrc* src,
                               const float* out, const float* y, const float* mean, const float* invstd,
                               const float* gamma, float* dgamma, float* dbeta, float* dy, tspm_stream_t stream);
int tspm_bn_bwd_apply_part(int64_t m, int32_t c, int32_t tiles, const float* part, const float* g, const float* out,
                           const float* y, const float* mean, const float* invstd, const float* gamma, float* dgamma,
                           float* dbeta, float* dy, const float* y2, const float* mean2, const float* invstd2,
                           const float* gamma2, float* dgamma2, float* dbeta2, float* dy2, float* dres,
                           tspm_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * Layout / data-stage helpers (collate → device, MML_Suite/data/avmnist.py:186-191,248-277)
 * ----------------------------------------------------------------------------------------------*/
/* image_f32[i] = lut[u8[i]] * (1/255)  (gist_earth→L colormap LUT, torchvision ToDtype(scale)). */
int tspm_image_lut(int64_t count, const uint8_t* u8, const uint8_t* lut, float* out, tspm_stream_t stream);
/* Batch assembly from an HBM-resident AVMNIST corpus (replaces, per batch, AVMNIST.__getitem__ +
 * _load_audio/_load_image + get_samples + collate_fn: MML_Suite/data/avmnist.py:164-224,248-277,
 * data/base_dataset.py:61-74).  For r < count, s = index[r]:
 *   audio_out[r,:]  = audio[s,:] * audio_mask[r]                       (audio_elems floats/row)
 *   image_out[r,:]  = (float)lut[image[s,:]] * fp32(1/255) * image_mask[r]  (image_elems bytes/row)
 *   labels_out[r]   = labels[s]
 * A null mask means "no multiply"; a null lut means the identity map; a null output skips that
 * modality (target_modality audio / image only).  An index outside [0, n_samples) writes NaN rows
 * and label -1 (tspm_cross_entropy then yields NaN) instead of reading out of bounds.
 * Fast path (16-byte audio, 4-byte image accesses) when both element counts are multiples of 4 and
 * audio/audio_out/image_out are 16-byte and image/lut 4-byte aligned; otherwise per element. */
int tspm_avmnist_gather(int64_t count, const int64_t* index, int64_t n_samples, const float* audio,
                        int32_t audio_elems, const uint8_t* image, int32_t image_elems, const int64_t* labels,
                        const uint8_t* lut, const float* audio_mask, const float* image_mask, float* audio_out,
                        float* image_out, int64_t* labels_out, tspm_stream_t stream);
/* Classification bookkeeping for one batch, on device (replaces the per-batch softmax → argmax →
 * .cpu() → MetricRecorder.update_group_all of models/avmnist.py:305-309,345-350 and
 * experiment_utils/metric_recorder.py:96-145, and the epoch loops' per-batch loss lists,
 * train_multimodal.py:478-491,525-541).  For r < n:
 *   pred = first argmax of softmax(logits[r,:classes]);  pred_out[r] = pred  (if pred_out)
 *   confusion[g][labels[r]][pred] += 1  with g = groups ? groups[r] : 0  (int64 counts,
 *   [n_groups][classes][classes]; rows whose label or group is out of range are not counted)
 * and once per call, when counters is given: loss_log[counters[0]] = *loss (if loss_log and
 * counters[0] < log_capacity), counters[0] += 1, counters[1] += n.  Graph-capturable. */
int tspm_classify_update(int32_t n, int32_t classes, const float* logits, const int64_t* labels,
                         const int32_t* groups, int32_t n_groups, int64_t* confusion, int64_t* pred_out,
                         const float* loss, float* loss_log, int64_t* counters, int64_t log_capacity,
                         tspm_stream_t stream);
/* Argmax conventions: the fusion model predicts argmax(softmax(logits)) (models/avmnist.py:305-306),
 * the monomodal pre-training step argmax(logits) (train_monomodal.py:236,394); they differ only when
 * two logits round to one probability. */
#define TSPM_ARGMAX_SOFTMAX 0
#define TSPM_ARGMAX_LOGITS 1
/* tspm_classify_update with an explicit convention (argmax_of: TSPM_ARGMAX_*). */
int tspm_classify_update_ex(int32_t n, int32_t classes, const float* logits, const int64_t* labels,
                            const int32_t* groups, int32_t n_groups, int64_t* confusion, int64_t* pred_out,
                            const float* loss, float* loss_log, int64_t* counters, int64_t log_capacity,
                            int32_t argmax_of, tspm_stream_t stream);
/* Sum `nslab` slabs of `count` floats (slab_stride apart) into out (deterministic slab order). */
int tspm_reduce_slabs(int64_t count, int32_t nslab, int64_t slab_stride, const float* slabs, float* out,
                      tspm_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * MMIMDb late-fusion path (BASELINE configs[3]; ABI 11).  The encoders (BatchNorm1d + Linear,
 * models/mmimdb.py:63-93) and the MaxOut / output projections reuse tspm_bn_* (m = batch rows, HW = 1)
 * and tspm_linear_*; these entry points add the pieces around them.
 * ----------------------------------------------------------------------------------------------*/
/* GatedBiModalNetwork.forward (models/gates/gated_bimodal.py): u[n,2d] holds fc_one(x1) in columns
 * [0,d) and fc_two(x2) in [d,2d).  h = tanh(u) (the concatenated features, [n,2d], kept for the
 * backward), gate[r] = sigmoid(sum_j wz[j]*h[r,j]) (hidden_sigmoid, no bias),
 * z[r,j] = gate*h[r,j] + (1-gate)*h[r,d+j]. */
int tspm_gmu_fwd(int32_t n, int32_t d, const float* u, int32_t ldu, const float* wz, float* h, int32_t ldh,
                 float* gate, float* z, int32_t ldz, tspm_stream_t stream);
/* Backward of tspm_gmu_fwd: du[n,2d] (gradient of both projections' outputs) and ds[n] (gradient of
 * the gate pre-activation; hidden_sigmoid.weight.grad = ds^T @ h via tspm_linear_bwd_weight). */
int tspm_gmu_bwd(int32_t n, int32_t d, const float* dz, int32_t lddz, const float* h, int32_t ldh,
                 const float* gate, const float* wz, float* du, int32_t lddu, float* ds, tspm_stream_t stream);
/* MultimodalPooling (ABI 13; models/pooling.py:6-127), the MMIMDb `multimodal_pooling` fusion.
 * u = [proj_a(x_a) | proj_b(x_b)] [n, 2d] from the small GEMM (with biases).
 * tspm_pool_act_fwd: tu = tanh(u), ab = tu * keep * keep_scale ([n, 2d] contiguous; keep nullable =
 *   no dropout; the module's one Dropout draws a and b independently).
 * tspm_pool_mix_fwd: z = max(a, b) (kind 0, NaN-propagating) / (a + b) / 2 (1) / a + b (2) /
 *   attention (3: w = softmax(W2 tanh(hpre) + b2), z = w0 a + w1 b) / gated (4: g = sigmoid(W2
 *   tanh(hpre) + b2), z = g a + (1 - g) b); hpre [n, hd] = the scoring MLP's first Linear (+ bias) of
 *   [a | b] (small GEMM); hh receives tanh(hpre), wts [n][2] the mixing weights (kinds 3-4).
 * tspm_pool_mix_bwd: dab [n, 2d] through the mix (max: ties split the gradient in half, as torch.maximum);
 *   kinds 3-4 also ds [n, 2 | 1] (scores' gradient: W2 grad = ds^T hh, b2 grad = column sums) and
 *   dhpre [n, hd] (through W2 and the tanh).
 * tspm_pool_act_bwd: du = (dab + dab2) * keep * keep_scale * (1 - tu^2) (dab2 nullable: the scoring
 *   MLP's input gradient). */
int tspm_pool_act_fwd(int32_t n, int32_t d, const float* u, int32_t ldu, const uint8_t* keep, float keep_scale,
                      float* tu, float* ab, tspm_stream_t stream);
int tspm_pool_mix_fwd(int32_t n, int32_t d, int32_t hd, int32_t kind, const float* ab, const float* hpre, float* hh,
                      const float* w2, const float* b2, float* wts, float* z, int32_t ldz, tspm_stream_t stream);
int tspm_pool_mix_bwd(int32_t n, int32_t d, int32_t hd, int32_t kind, const float* dz, int32_t lddz, const float* ab,
                      const float* hh, const float* w2, const float* wts, float* dab, float* ds, float* dhpre,
                      tspm_stream_t stream);
int tspm_pool_act_bwd(int32_t n, int32_t d, const float* dab, const float* dab2, const float* tu, const uint8_t* keep,
                      float keep_scale, float* du, tspm_stream_t stream);
/* MaxOut(num_units=2) (models/maxout.py) + the Dropout after it (models/mmimdb.py:40-45): a[n,2d] is
 * the product with both units' weights stacked ([2d, in] — layers.0.weight then layers.1.weight);
 * y = max(a[:, :d], a[:, d:]) * (keep ? keep_scale : 0)  (keep NULL: no dropout). */
int tspm_maxout_fwd(int32_t n, int32_t d, const float* a, int32_t lda, const uint8_t* keep, float keep_scale,
                    float* y, int32_t ldy, tspm_stream_t stream);
/* tspm_maxout_fwd with the dropout mask drawn in-launch (ABI 11): keep[t] = the bit tspm_dropout_mask(
 * count, p, seed, counter) writes at index index_offset + t (stored for the backward), y as tspm_maxout_fwd
 * with that mask — one launch instead of mask + MaxOut. */
int tspm_maxout_fwd_rng(int32_t n, int32_t d, const float* a, int32_t lda, float p, uint64_t seed,
                        const uint64_t* counter, int64_t index_offset, uint8_t* keep, float keep_scale, float* y,
                        int32_t ldy, tspm_stream_t stream);
/* da[n,2d] from dy: the unit holding the max receives the (dropout-masked) gradient; ties split it in
 * half (ATen's derivative of torch.maximum). */
int tspm_maxout_bwd(int32_t n, int32_t d, const float* dy, int32_t lddy, const float* a, int32_t lda,
                    const uint8_t* keep, float keep_scale, float* da, int32_t ldda, tspm_stream_t stream);
/* BatchNorm1d, training mode, over x[m, c] (m = batch rows; models/mmimdb.py:78,38-46), in one launch:
 * batch mean / biased variance for y = gamma*(x-mean)*invstd + beta, running statistics updated with
 * the unbiased variance (momentum, eps as nn.BatchNorm1d; NULL running buffers skip the update),
 * save_mean / save_invstd [c] kept for the backward.  No workspace. */
int tspm_bn1d_fwd(int32_t m, int32_t c, const float* x, const float* gamma, const float* beta,
                  float* running_mean, float* running_var, float momentum, float eps, float* save_mean,
                  float* save_invstd, float* y, tspm_stream_t stream);
/* Its backward in one launch: dgamma = sum(g*xhat), dbeta = sum(g) (written), and (dx nullable)
 * dx = gamma*invstd*(g - dbeta/m - xhat*dgamma/m). */
int tspm_bn1d_bwd(int32_t m, int32_t c, const float* g, const float* x, const float* mean, const float* invstd,
                  const float* gamma, float* dgamma, float* dbeta, float* dx, tspm_stream_t stream);
/* BatchNorm1d followed by Dropout (FcClassifier(use_bn=True): Linear -> ReLU -> BatchNorm1d -> Dropout,
 * models/msa/networks/classifier.py:98-104; ABI 14): tspm_bn1d_fwd, then y *= keep ? keep_scale : 0
 * (keep uint8 [m, c], nullable = no dropout). */
int tspm_bn1d_fwd_drop(int32_t m, int32_t c, const float* x, const float* gamma, const float* beta,
                       float* running_mean, float* running_var, float momentum, float eps, float* save_mean,
                       float* save_invstd, const uint8_t* keep, float keep_scale, float* y, tspm_stream_t stream);
/* Its backward (ABI 14): g is the gradient of the Dropout output (g_keep nullable), x the BatchNorm input =
 * a ReLU output; dgamma / dbeta as tspm_bn1d_bwd on g*keep*g_scale, dx (nullable) = the BN input gradient
 * with the ReLU's mask applied (0 where x <= 0) — the gradient of the Linear that fed the ReLU. */
int tspm_bn1d_bwd_drop_relu(int32_t m, int32_t c, const float* g, const uint8_t* g_keep, float g_scale,
                            const float* x, const float* mean, const float* invstd, const float* gamma,
                            float* dgamma, float* dbeta, float* dx, tspm_stream_t stream);
/* Two independent BatchNorm1d layers over the same m rows in one launch (the MMIMDb image and text
 * encoders' input BNs; ABI 11): each half exactly as tspm_bn1d_fwd / tspm_bn1d_bwd (bitwise). */
int tspm_bn1d_fwd_pair(int32_t m, int32_t c0, const float* x0, const float* gamma0, const float* beta0,
                       float* running_mean0, float* running_var0, float momentum0, float eps0, float* save_mean0,
                       float* save_invstd0, float* y0, int32_t c1, const float* x1, const float* gamma1,
                       const float* beta1, float* running_mean1, float* running_var1, float momentum1, float eps1,
                       float* save_mean1, float* save_invstd1, float* y1, tspm_stream_t stream);
int tspm_bn1d_bwd_pair(int32_t m, int32_t c0, const float* g0, const float* x0, const float* mean0,
                       const float* invstd0, const float* gamma0, float* dgamma0, float* dbeta0, float* dx0,
                       int32_t c1, const float* g1, const float* x1, const float* mean1, const float* invstd1,
                       const float* gamma1, float* dgamma1, float* dbeta1, float* dx1, tspm_stream_t stream);
/* BCEWithLogitsLoss (mean) — LossFunctionGroup{bce_with_logits: w} (experiment_utils/loss.py:52,
 * configs/mmimdb/centralised/mmimdb_baseline.yaml): loss[0] = grad_scale * mean((1-t)*x - logsigmoid(x)),
 * dlogits = (sigmoid(x) - t) * grad_scale / (n*classes) (nullable).  If stats != NULL (3 + 3*classes
 * floats, accumulated): [0] += loss*n, [1] += n, [2] += sum of per-sample F1 (zero_division 0),
 * [3+3k .. 5+3k] += tp, fp, fn of class k, with prediction = sigmoid(x) > threshold
 * (models/mmimdb.py:236-237). */
int tspm_bce_logits(int32_t n, int32_t classes, const float* logits, const float* targets, float* loss,
                    float* dlogits, float grad_scale, float threshold, float* stats, tspm_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * MOSI UTT-Fusion (BASELINE configs[4]; ABI 12) — MML_Suite/models/msa/utt_fusion.py:25-200 with
 * configs/mosi/centralised/utt_fusion_base_training.yaml.  Sequences are time-major on the device:
 * row (t, b) of a [T][B][F] tensor.
 * ----------------------------------------------------------------------------------------------*/
/* nn.LSTM(input, hidden, batch_first=True), one layer, zero initial state, embd_method "last" or
 * "maxpool" (models/msa/networks/lstm.py:8-67; the reference runs the padded length, no packing).
 * xg = x W_ih^T + b_ih for all steps (a tspm_linear_fwd over the T*B rows); the recurrence adds
 * h W_hh^T + b_hh.  Saved for the backward: activated gates i,f,g,o [T][B][4H], c_t [T][B][H], h_t
 * [T+1][B][H] (hs[0] = h0 = 0).  argmax NULL ("last"): h_T goes to h_out (row stride ld_out); argmax
 * non-NULL ("maxpool", ABI 14; lstm.py:47-52 F.max_pool1d over r_out): max over t of h_t goes to h_out
 * and its time index (first maximum, NaN wins) to argmax uint8 [batch][hidden] (steps <= 256).  hidden
 * must be 64; any batch >= 1 (an odd batch leaves the last 2-row workgroup one ghost row, which reads the
 * last real row and writes nothing). */
typedef struct tspm_lstm_fwd_desc {
  int32_t batch, steps, hidden, ld_out;
  const float* xg;
  const float* w_hh;
  const float* b_hh; /* nullable */
  float* gates;
  float* cs;
  float* hs;
  float* h_out;
  uint8_t* argmax; /* nullable; ABI 14 */
} tspm_lstm_fwd_desc;
/* 1 or 2 independent LSTMs (the audio and video encoders) in one launch. */
int tspm_lstm_fwd(int32_t count, const tspm_lstm_fwd_desc* descs, tspm_stream_t stream);
/* Backward through time from dh (the gradient of the embedding, row stride ld_dh: of h_T, or with
 * argmax (ABI 14) of h_{argmax} per unit, the max-pool backward): writes the pre-activation
 * gate gradients dgates [T][B][4H].  The weight gradients are then GEMMs over the T*B rows:
 * dW_hh = dgates^T hs[0:T], dW_ih = dgates^T x, db_hh = db_ih = column sums of dgates. */
typedef struct tspm_lstm_bwd_desc {
  int32_t batch, steps, hidden, ld_dh;
  const float* w_hh;
  const float* gates;
  const float* cs;
  const float* dh;
  float* dgates;
  const uint8_t* argmax; /* nullable; ABI 14 */
} tspm_lstm_bwd_desc;
int tspm_lstm_bwd(int32_t count, const tspm_lstm_bwd_desc* descs, tspm_stream_t stream);
/* TextCNN pooling (models/msa/networks/textcnn.py:56-67): for conv i (kernel height heights[i], output
 * conv_out[i] time-major [steps-heights[i]+1][batch][channels] without bias), bias[i] added, ReLU,
 * max over time (first maximum, F.max_pool1d), concatenated over convs: pooled[b][i*C+c] and the
 * argmax time index; out[b*ld_out + i*C+c] = pooled * (keep ? keep*keep_scale : 1) — the dropout before
 * the embedding Linear (keep uint8 [batch][nconv*C], nullable).  nconv <= 4, steps <= 256. */
int tspm_textcnn_pool_fwd(int32_t batch, int32_t steps, int32_t nconv, const int32_t* heights,
                          int32_t channels, const float* const* conv_out, const float* const* bias,
                          const uint8_t* keep, float keep_scale, float* pooled, uint8_t* argmax,
                          float* out, int32_t ld_out, tspm_stream_t stream);
/* TextCNN backward from dout (gradient of the embedding Linear's input, row stride ld_dout): through the
 * dropout and the ReLU at the argmax; conv weight gradients dw[i] ([C][heights[i]][feat], the
 * nn.Conv2d(1, C, (h, feat)) weight layout) and bias gradients db[i] (nullable) from the argmax rows
 * only (the time-max passes gradient to one position per (b, c)): dw[c][dt][f] = sum_b g[b][c]
 * x[arg[b][c] + dt][b][f].  x is the time-major text input [steps][batch][feat] (feat <= 1024,
 * heights <= 5); g_work holds batch*nconv*channels floats. */
int tspm_textcnn_bwd(int32_t batch, int32_t steps, int32_t feat, int32_t nconv, const int32_t* heights,
                     int32_t channels, const float* x, const float* dout, int32_t ld_dout, const uint8_t* keep,
                     float keep_scale, const float* pooled, const uint8_t* argmax, float* const* dw,
                     float* const* db, float* g_work, tspm_stream_t stream);
/* clip_grad_norm_(parameters, max_norm) coefficient (utt_fusion.py:189): total = ||grad * grad_scale||_2
 * (squares summed in double, fixed order), *coef = min(1, max_norm / (total + 1e-6)) for
 * tspm_adam_step_clip; *total_norm (nullable) = total.  workspace: tspm_grad_clip_workspace() bytes. */
size_t tspm_grad_clip_workspace(void);
int tspm_grad_clip_coef(int64_t count, const float* grad, float grad_scale, float max_norm, float* coef,
                        float* total_norm, void* workspace, size_t workspace_bytes, tspm_stream_t stream);
/* Padded batch assembly (data/mosi.py:202-232 pad_sequence + the step's .to(device)) from a ragged
 * corpus data[rows][feat] (sample s = rows offsets[s] .. offsets[s]+lengths[s]-1): out[t*stride_t +
 * b*stride_b + f] = sample index[b]'s row t (0 past its length) * row_mask[b] (nullable), for
 * t < steps_pad; labels_out[b] = labels[index[b]] (both nullable).  Out-of-range indices write NaN
 * rows and label -1. */
int tspm_seq_gather(int32_t count, const int64_t* index, int64_t n_samples, const float* data,
                    const int64_t* offsets, const int32_t* lengths, int32_t feat, int32_t steps_pad, float* out,
                    int64_t stride_t, int64_t stride_b, const float* row_mask, const int64_t* labels,
                    int64_t* labels_out, tspm_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* TSPM_H_ */
