/*
 * zenflow_amd.h — C ABI of the MI355X-native zenflow hot path (libzenflow_amd.so).
 *
 * The reference (HDembinski/zenflow, a JAX/FLAX library) has no FFI: its
 * boundary is the FLAX module protocol.  Each entry point below replaces one
 * reference callable (cited file:line, relative to the reference repo); the
 * Python package `zenflow_amd` binds them with ctypes and re-exposes the
 * reference's names and signatures (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - Plain pointers and sizes only.  Device pointers come from zf_malloc (or
 *     any hipMalloc'ed buffer); `stream` is a hipStream_t passed as void*
 *     (NULL = the legacy default stream).
 *   - Every function returns 0 on success, a negative ZF_E* code on a bad
 *     argument, or a positive hipError_t.  zf_last_error() returns a
 *     thread-local message for the last failure.
 *   - All floating-point data is fp32, row-major; log-det / NLL partial sums
 *     are fp64.  Kernels never trap on NaN/Inf: they propagate exactly as the
 *     reference does.
 */
#ifndef ZENFLOW_AMD_H
#define ZENFLOW_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZF_OK 0
#define ZF_EINVAL (-1)     /* invalid argument / shape */
#define ZF_ENOTSUP (-2)    /* configuration not supported by the kernels */
#define ZF_ENOMEM (-3)

/* ------------------------------------------------------------------------ */
/* Runtime: devices, memory, streams, events (plumbing for the host layer).  */
/* ------------------------------------------------------------------------ */
const char* zf_last_error(void);
int zf_version(void);
int zf_device_count(int* count);
int zf_set_device(int device);
int zf_get_device(int* device);
int zf_device_name(int device, char* buf, int buflen);
int zf_device_synchronize(void);
int zf_malloc(void** ptr, size_t bytes);
int zf_free(void* ptr);
int zf_memset_async(void* ptr, int value, size_t bytes, void* stream);
/* Host <-> device copies, ordered on `stream`.  htod returns once `src` may be
 * reused (the copy itself completes in stream order); dtoh returns with `dst`
 * filled (up to 4 MiB through a pinned staging buffer). */
int zf_memcpy_htod(void* dst, const void* src, size_t bytes, void* stream);
int zf_memcpy_dtoh(void* dst, const void* src, size_t bytes, void* stream);
int zf_memcpy_dtod(void* dst, const void* src, size_t bytes, void* stream);
int zf_stream_create(void** stream);
int zf_stream_destroy(void* stream);
int zf_stream_synchronize(void* stream);
int zf_event_create(void** event);
int zf_event_destroy(void* event);
int zf_event_record(void* event, void* stream);
int zf_event_elapsed_ms(void* start, void* stop, float* ms);
int zf_event_synchronize(void* event);
/* Work queued on `stream` after this call waits for `event` (hipStreamWaitEvent). */
int zf_stream_wait_event(void* stream, void* event);

/* ------------------------------------------------------------------------ */
/* K1 — spline numerics at the `zenflow.utils` boundary.                     */
/* ------------------------------------------------------------------------ */
/* Replaces utils.rational_quadratic_spline_forward (src/zenflow/utils.py:65-141).
 * x (M,N), dx/dy (M,N,K) normalised widths/heights, slope (M,N,K-1) inner knot
 * derivatives -> y (M,N), log_det (M,) = sum over N of log dy/dx.
 * y and/or log_det may be NULL. */
int zf_rqs_forward(const float* x, const float* dx, const float* dy, const float* slope,
                   float* y, float* log_det, int64_t M, int N, int K, void* stream);

/* Replaces utils.rational_quadratic_spline_inverse (src/zenflow/utils.py:144-202). */
int zf_rqs_inverse(const float* y, const float* dx, const float* dy, const float* slope,
                   float* x, int64_t M, int N, int K, void* stream);

/* Replaces utils.squareplus (src/zenflow/utils.py:18-20), elementwise, b = 4 by default. */
int zf_squareplus(const float* x, float* y, int64_t n, float b, void* stream);

/* Replaces utils.softmax_with_threshold (src/zenflow/utils.py:23-34) over rows of K. */
int zf_softmax_with_threshold(const float* x, float* y, int64_t M, int K, double threshold,
                              void* stream);

/* Replaces utils.normalize_spline_params (src/zenflow/utils.py:37-62):
 * raw (M, K) / (M, K) / (M, K-1) logits -> normalised, written in place. */
int zf_normalize_spline_params(float* dx, float* dy, float* slope, int64_t M, int K,
                               void* stream);

/* ------------------------------------------------------------------------ */
/* Fused flow program: ShiftBounds / NeuralSplineCoupling / Roll / latent.   */
/* ------------------------------------------------------------------------ */

/* Op kinds of a flow program (one per reference bijector). */
#define ZF_OP_SHIFT_BOUNDS 1 /* bijectors.ShiftBounds         bijectors.py:132-273 */
#define ZF_OP_ROLL 2         /* bijectors.Roll                bijectors.py:276-297 */
#define ZF_OP_NSC 3          /* bijectors.NeuralSplineCoupling bijectors.py:300-371 */

/* Latent log_prob epilogues (distributions.py). */
#define ZF_LATENT_NONE 0
#define ZF_LATENT_NORMAL 1    /* distributions.py:50-62  */
#define ZF_LATENT_BETA 2      /* distributions.py:81-116 */
#define ZF_LATENT_TRUNCNORM 3 /* distributions.py:65-78  */
#define ZF_LATENT_UNIFORM 4   /* distributions.py:119-126 */

/* Activation of the conditioner's hidden layers (NSC.act, bijectors.py:319;
 * the flax.linen / jax.nn functions of those names).  Split-MFMA kernel
 * (zf_flow_kernel_variant): all eight on the f16x2 scheme (sigmoid and
 * softplus centred on 1/2 and log 2); under ZF_X3_SCHEME=bf16x3 softplus
 * runs on the fp32 kernel.  The trainer takes all eight. */
#define ZF_ACT_SWISH 0      /* nn.swish = nn.silu: x * sigmoid(x) */
#define ZF_ACT_RELU 1       /* nn.relu */
#define ZF_ACT_TANH 2       /* nn.tanh */
#define ZF_ACT_SIGMOID 3    /* nn.sigmoid */
#define ZF_ACT_GELU 4       /* nn.gelu (approximate=True, the flax default) */
#define ZF_ACT_SOFTPLUS 5   /* nn.softplus = logaddexp(x, 0) */
#define ZF_ACT_ELU 6        /* nn.elu (alpha 1) */
#define ZF_ACT_LEAKY_RELU 7 /* nn.leaky_relu (negative slope 0.01) */
#define ZF_ACT_COUNT 8

/* ShiftBounds per-dim modes (bijectors.py:183-205). */
#define ZF_SB_NONE 0  /* unbounded: running min/max affine + clip        */
#define ZF_SB_BOTH 1  /* (a, b) both finite: fixed affine                */
#define ZF_SB_LOWER 2 /* only a: t = safe_log(x - a), then min/max affine */
#define ZF_SB_UPPER 3 /* only b: t = safe_log(b - x), then min/max affine */

typedef struct zf_op_desc {
  int32_t kind;       /* ZF_OP_* */
  /* ROLL */
  int32_t shift;      /* jnp.roll shift along the last axis */
  /* NSC */
  int32_t knots;      /* K (2 <= K <= 64) */
  int32_t n_hidden;   /* number of hidden Dense layers (len(layers)), 1..16 */
  int32_t hidden[16]; /* widths of the hidden layers (each <= 4096; > 256: the layered path) */
  int32_t act;        /* ZF_ACT_* */
  int32_t _pad;
  /* Offsets (in floats) into the NATURAL parameter blob, filled by
   * zf_flow_plan.  The natural blob holds exactly the FLAX variables:
   *   NSC:  off_bn -> BatchNorm_0 {mean[DC], var[DC], scale[DC], bias[DC]}
   *         (DC = D - D/2 + C conditioner inputs),
   *         off_w[l] -> Dense_l.kernel, row-major (in_l, out_l),
   *         off_b[l] -> Dense_l.bias (out_l); l = 0..n_hidden, the last layer
   *         has out = (D/2)*(3K-1) (bijectors.py:343-347).
   *   SHIFT_BOUNDS: off_sb -> per dim 8 floats {mode(ZF_SB_*), a, b, xmin, xmax, 0, 0, 0}
   *         (batch_stats xmin_i / xmax_i, bijectors.py:243-248). */
  int64_t off_bn;
  int64_t off_w[17];
  int64_t off_b[17];
  int64_t off_sb;
} zf_op_desc;

typedef struct zf_flow_desc {
  int32_t dim;        /* D: data dims (2..64 when the flow has an NSC) */
  int32_t cond_dim;   /* C: condition dims (0 = unconditional) */
  int32_t latent;     /* ZF_LATENT_* */
  float latent_param; /* Beta peakness */
  int32_t n_ops;      /* <= 64 */
  int32_t _pad;
  zf_op_desc ops[64];
} zf_flow_desc;

typedef struct zf_flow zf_flow_t; /* opaque handle: device-resident packed weights */

/* Validate `desc` and fill its natural-blob offsets; *blob_floats = size of
 * the natural blob.  Host-side only. */
int zf_flow_plan(zf_flow_desc* desc, int64_t* blob_floats);

/* Pack the natural blob into the device layout (MFMA fragment order, BN
 * folded to (mean, rsqrt(var+eps)*scale, bias), ShiftBounds mul/log(mul))
 * and copy it to the current device.  The handle owns the device copy until
 * zf_flow_destroy. */
int zf_flow_create(const zf_flow_desc* desc, const float* blob_host, int64_t blob_floats,
                   zf_flow_t** handle);
int zf_flow_destroy(zf_flow_t* handle);

/* Which kernel the handle runs (no reference counterpart: an
 * implementation detail made observable for tests and benchmarks):
 * ZF_KERNEL_FP32 (fp32 MFMA, any shape up to hidden 256), the split-MFMA
 * kernel for the shapes it covers (x3_eligible: every hidden width <= 256,
 * one knot count in 2..32 for all couplings — 8, 16, 32 instantiated, the
 * others padded with inert knots, 31 excepted — dim <= 64) in one of two
 * schemes: ZF_KERNEL_F16X2 (default: two-term fp16 split of
 * power-of-two-scaled operands, three fp16 MFMAs per k-step) or
 * ZF_KERNEL_BF16X3 (three-term bf16 split, six bf16 MFMAs per k-step;
 * ZF_X3_SCHEME=bf16x3, where a softplus coupling runs on the fp32 kernel), or
 * ZF_KERNEL_LAYERED (a hidden width above 256: op by op).  The environment
 * is read at zf_flow_create time; ZF_DISABLE_X3=1 forces ZF_KERNEL_FP32 for
 * fused shapes.  -1 if h is NULL. */
#define ZF_KERNEL_FP32 0
#define ZF_KERNEL_BF16X3 1
#define ZF_KERNEL_F16X2 2
#define ZF_KERNEL_LAYERED 3 /* a hidden width > 256: op by op (BatchNorm, GEMMs, spline kernels) */
int zf_flow_kernel_variant(const zf_flow_t* h);

/* Device workspace needed by zf_flow_log_prob for N rows. */
int64_t zf_flow_workspace_bytes(int64_t N);

/* Replaces Flow.__call__ = log_prob (src/zenflow/flow.py:22-48), eval mode:
 * x (N,D), c (N,C) or NULL -> log_prob (N,) with NaN -> -inf, +-inf -> +-FLT_MAX
 * (jnp.nan_to_num, flow.py:47).  If nll_sum != NULL, the per-block fp64
 * partial sums of log_prob are reduced on device into nll_sum[0]
 * (NLL = -nll_sum/N, train.py:75-78). */
int zf_flow_log_prob(zf_flow_t* h, const float* x, const float* c, float* log_prob,
                     double* nll_sum, void* workspace, int64_t N, void* stream);

/* Segment form of zf_flow_log_prob: runs ops [op_begin, op_end) on x, seeds
 * the log-det accumulator from log_det_in (may be NULL), then applies the
 * latent epilogue (train mode runs the bijectors segment by segment).  With a
 * workspace the kernel writes per-block fp64 partial sums of log_prob there;
 * with nll_sum it also reduces them (else call zf_flow_nll_reduce). */
int zf_flow_log_prob_segment(zf_flow_t* h, int op_begin, int op_end, const float* x,
                             const float* c, const float* log_det_in, float* log_prob,
                             double* nll_sum, void* workspace, int64_t N, void* stream);

/* Fixed-order fp64 sum of the per-block partials a log_prob launch left in
 * `workspace` for N rows -> nll_sum[0] (= sum log_prob; NLL = -nll_sum/N). */
int zf_flow_nll_reduce(const void* workspace, int64_t N, double* nll_sum, void* stream);

/* Replaces Chain.__call__ (bijectors.py:103-111) over the op range
 * [op_begin, op_end): x (N,D) -> y (N,D), log_det (N,).  If log_det_in is not
 * NULL its values seed the accumulator (chained segments, train mode). */
int zf_flow_forward(zf_flow_t* h, int op_begin, int op_end, const float* x, const float* c,
                    float* y, const float* log_det_in, float* log_det, int64_t N,
                    void* stream);

/* Replaces Chain.inverse (bijectors.py:113-116) / the bijector half of
 * Flow.sample (flow.py:70-78) over [op_begin, op_end), applied in reverse:
 * z (N,D) -> x (N,D). */
int zf_flow_inverse(zf_flow_t* h, int op_begin, int op_end, const float* z, const float* c,
                    float* x, int64_t N, void* stream);

/* Replaces Flow.sample (flow.py:50-78) end to end: the latent draw
 * (distributions.py:61-62 / 75-78 / 106-112 / 125-126) happens on the device
 * in the inverse kernel's prologue — Philox4x32-10 keyed by `seed`, counter =
 * (row, dim, stream), so x[row] depends only on (seed, row) — then the whole
 * Chain.inverse runs in the same launch.  c (N,C) or NULL -> x (N,D).
 * jax.random's threefry bits are not reproduced (parity is statistical). */
int zf_flow_sample(zf_flow_t* h, uint64_t seed, const float* c, float* x, int64_t N, void* stream);

/* Replaces Distribution.sample (distributions.py:61-62 Normal, :75-78
 * TruncatedNormal, :106-112 Beta(param, param), :125-126 Uniform): z (N,D)
 * drawn with the same counter-based generator as zf_flow_sample (same seed
 * -> the same z that zf_flow_sample maps through the inverse). */
int zf_latent_sample(int latent, double param, uint64_t seed, float* z, int64_t N, int D, void* stream);

/* Replace one NSC op's BatchNorm statistics (mean[DC], var[DC]) — flax
 * BatchNorm with use_running_average=False normalises by batch statistics. */
int zf_flow_set_bn_stats(zf_flow_t* h, int op, const float* mean, const float* var);

/* Replace one ShiftBounds op's per-dim xmin/xmax (bijectors.py:250-263). */
int zf_flow_set_sb_stats(zf_flow_t* h, int op, const float* xmin, const float* xmax);

/* ------------------------------------------------------------------------ */
/* Train-mode batch statistics (reductions over the batch axis).             */
/* ------------------------------------------------------------------------ */
/* Per column j (0 <= j < ncols) of x (N rows, row stride `ld` floats, first
 * column `col_offset`): min, max (fp32, NaN-propagating like jnp.min/max) and
 * sum, sum of squares (fp64).  ShiftBounds' batch min/max (bijectors.py:250-257)
 * and flax BatchNorm's batch mean/var (bijectors.py:342, train=True).
 * pre_modes/pre_params (host arrays of ncols, or NULL): per column ZF_SB_LOWER
 * -> safe_log(x - a), ZF_SB_UPPER -> safe_log(a - x) with a = pre_params[j]
 * (the one-sided-bound transform, bijectors.py:193-202).  Outputs are device
 * pointers (any may be NULL); workspace: zf_colstats_workspace_bytes(N, ncols). */
int64_t zf_colstats_workspace_bytes(int64_t N, int ncols);
int zf_colstats(const float* x, int64_t N, int ncols, int64_t ld, int col_offset,
                const float* pre_modes, const float* pre_params, float* cmin, float* cmax,
                double* csum, double* csumsq, void* workspace, void* stream);

/* ------------------------------------------------------------------------ */
/* Training — zenflow.train (src/zenflow/train.py:18-138).                    */
/* ------------------------------------------------------------------------ */

/* optax.adamw / optax.nadamw hyper-parameters (train.py:13-16 default:
 * nadamw(learning_rate=1e-3); optax defaults b1 0.9, b2 0.999, eps 1e-8,
 * weight_decay 1e-4). */
typedef struct zf_optim_desc {
  float learning_rate, b1, b2, eps, weight_decay;
  int nesterov; /* 1: nadamw, 0: adamw */
} zf_optim_desc;

typedef struct zf_trainer zf_trainer_t;

/* A trainer owns a device copy of the natural blob (zf_flow_plan layout:
 * parameters AND batch statistics), its gradient and the optimiser moments.
 * param_mask[i] = 1 marks the blob entries that are parameters (updated by
 * the optimiser), 0 the batch statistics.  ShiftBounds rows carry the margin
 * in slot 5.  ShiftBounds is supported as the first op only; conditioner
 * inputs <= 64; batches up to batch_max rows. */
int zf_trainer_create(const zf_flow_desc* desc, const float* blob_host, int64_t blob_floats,
                      const unsigned char* param_mask, int64_t batch_max, const zf_optim_desc* opt,
                      zf_trainer_t** trainer);
int zf_trainer_destroy(zf_trainer_t* trainer);

/* loss_fn of train.py:64-72 and its gradient (jax.grad): train-mode forward
 * (batch statistics) of x (B,D), c (B,C) or NULL on the device; loss[0] (fp64,
 * device) = -mean(log_prob); grad (device, blob layout; NULL: internal) =
 * d loss / d blob (zero on statistics).  update_stats != 0 also applies the
 * running-statistics updates (ShiftBounds min/max, BatchNorm momentum). */
int zf_trainer_loss_grad(zf_trainer_t* trainer, const float* x, const float* c, int64_t B, int update_stats,
                         double* loss, float* grad, void* stream);

/* step of train.py:80-86: loss_grad with statistics update, then the
 * optimiser update of the parameters. */
int zf_trainer_step(zf_trainer_t* trainer, const float* x, const float* c, int64_t B, double* loss,
                    void* stream);

/* Data-parallel training: one trainer per GPU, each
 * on its shard of every global batch.  The trainer exchanges at every batch
 * reduction of loss_fn and its gradient — the ShiftBounds batch min/max
 * (bijectors.py:250-257), the BatchNorm batch sums forward and reverse
 * (bijectors.py:342, flax BatchNorm), the loss (train.py:64-72) and the
 * gradient (train.py:82) — through one primitive:
 *   allgather(ctx, send, recv, bytes, stream): recv[world][bytes] = every
 *   rank's `bytes` of send, in rank order, ordered on `stream`
 * (zf_rccl_allgather with ctx = an RCCL communicator, or any host transport
 * that completes it synchronously).  Every sum is a fixed tree over row
 * leaves whose count depends on the global batch only, and the ranks combine
 * their subtree roots by the top of that tree: every rank gets the same
 * bits, and R ranks (a power of two, equal shards) the bits one device gets
 * on the whole batch.  NULL / world 1: single device (the default). */
typedef int (*zf_allgather_fn)(void* ctx, const void* send, void* recv, size_t bytes, void* stream);
typedef struct zf_comm_desc {
  int rank, world;
  void* ctx;
  zf_allgather_fn allgather;
} zf_comm_desc;
int zf_trainer_set_comm(zf_trainer_t* trainer, const zf_comm_desc* comm);

/* loss_grad / step on this rank's `rows` rows of a global batch of
 * `global_rows` rows (the loss is -mean over the global batch; the gradient
 * and loss returned are the global ones, identical on every rank).  The
 * plain entries above use global_rows = rows * world. */
int zf_trainer_loss_grad_shard(zf_trainer_t* trainer, const float* x, const float* c, int64_t rows,
                               int64_t global_rows, int update_stats, double* loss, float* grad, void* stream);
int zf_trainer_step_shard(zf_trainer_t* trainer, const float* x, const float* c, int64_t rows, int64_t global_rows,
                          double* loss, void* stream);

/* Copy the trainer's natural blob (parameters + statistics) out / in. */
int zf_trainer_get_blob(zf_trainer_t* trainer, float* blob_host);
int zf_trainer_set_blob(zf_trainer_t* trainer, const float* blob_host);

/* ------------------------------------------------------------------------ */
/* RCCL (over xGMI) — the NLL all-reduce of data-parallel log_prob and the  */
/* trainer's all-gather.                                                      */
/* ------------------------------------------------------------------------ */
int zf_rccl_available(void);
int zf_rccl_get_unique_id(char* id128);
int zf_rccl_comm_init(void** comm, int nranks, const char* id128, int rank);
int zf_rccl_allreduce_sum_f64(void* comm, const double* send, double* recv, size_t count,
                              void* stream);
int zf_rccl_comm_destroy(void* comm);
/* zf_allgather_fn over RCCL (ncclAllGather of bytes): comm = ctx. */
int zf_rccl_allgather(void* comm, const void* send, void* recv, size_t bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ZENFLOW_AMD_H */
