/*
 * vae2_hip.h — C ABI of libvae2_hip.so, the MI355X (gfx950) kernels of the VAE²
 * ELBO training step.
 *
 * The reference has no FFI: its hot path is Python calling ATen.
 * Every entry point below replaces one ATen op class used by that path; the
 * reference call site it stands in for is cited per function.
 *
 * Conventions
 *   - Stateless launchers over CALLER-OWNED device buffers. The library never
 *     allocates device memory; workspaces are sized by the *_size / *_rows queries.
 *   - Activations are NHWC fp32 views described by vae2_act:
 *        element (n, y, x, c) lives at ptr[((n*h + y)*w + x)*ps + c],  ps >= c.
 *     A channel slice of a wider buffer is (ptr + c0, ps = width of the buffer).
 *   - Conv weights keep the reference's nn.Conv2d layout [Cout][Cin][KH][KW]
 *     (so state_dicts interchange); conv biases are [Cout].
 *   - `stream` is a hipStream_t (PyTorch: torch.cuda.current_stream().cuda_stream).
 *   - Return 0 on success, a hipError_t value on a launch error, or -22 (EINVAL)
 *     for a bad argument; vae2_last_error() gives the message (thread-local).
 */
#ifndef VAE2_HIP_H
#define VAE2_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vae2_act {
  int64_t n, h, w, c;
  int64_t ps; /* pixel stride, in elements */
} vae2_act;

#define VAE2_ABI_VERSION 12

int vae2_abi_version(void);
const char* vae2_last_error(void);

/* Kernel launch log for profilers (bench.py's live per-kernel table): with logging
 * enabled every kernel the calling thread launches is recorded; _read returns how
 * many were launched since the last read and writes their names (as rocprofv3 shows
 * them, without "vae2::" and the parameter list, ';'-separated) into buf.  Enabling
 * or disabling clears the log.                                                    */
int vae2_kernel_log(int enable);
int64_t vae2_kernel_log_read(char* buf, int64_t len);

/* ---------------------------------------------------------------- conv ---- */

/* Rows of BN partial statistics that vae2_conv2d_fwd writes when stats != NULL
 * (one row of `cout` sums and one of `cout` sums of squares per row), for this
 * input (its address decides which kernel runs), geometry and output.
 * Workspace = 2 * rows * cout floats.                                         */
int64_t vae2_conv2d_fwd_stats_rows(const float* x, const vae2_act* xd, const vae2_act* yd,
                                   int k, int stride, int pad);

/* Conv algorithm selection (tuning / A-B measurement): 0 = auto, 1 = the gather
 * implicit-GEMM kernel only, 2 = the LDS-tiled direct 3x3 kernel wherever legal
 * (k = 3, stride 1, pad 1, 16-byte aligned input with ps % 4 == 0); + 4 also
 * disables the wide-N tiles of 1x1 convs, + 8 the in-workgroup K split of the
 * implicit-GEMM kernel for layers with few row tiles, + 16 the VALU-remainder channels of
 * the direct 3x3 kernels (18 = 16 + 2 ...), + 32 the persistent 1x1 GEMM, + 64 the
 * quad-transposed 16-byte epilogue stores / operand loads, + 128 the 32 + 4 and 64 + 8
 * remainder forms in auto mode.  Returns the previous setting.
 * Process-wide; set it before building stats buffers.                           */
int vae2_conv2d_set_algo(int algo);
/* MFMA operand precision of every conv kernel (forward, data and weight gradient):
 * 0 = fp32 operands (v_mfma_f32_16x16x4_f32, exact fp32 products; the default),
 * 1 = bf16 operands (v_mfma_f32_16x16x32_bf16: activations, gradients and weights are
 * rounded to bf16 (RNE) as they enter the MFMA; accumulation, storage, BatchNorm and the
 * optimizer stay fp32).  Returns the previous setting.  Process-wide.             */
int vae2_conv2d_set_mfma_bf16(int on);
/* Launch-shape tuning knobs for A/B measurements (every setting computes the same
 * result): key 0 = minimum igemm workgroups (row tiles shrink 4 -> 2 -> 1 until the grid
 * reaches it; default 512, 0 = the 4-row-tile rule alone); key 1 = 1: weight gradients with 64 (tap, Cin4)
 * columns take 2 x 16 output-channel rows and all 64 columns per workgroup (not 4 x 16
 * rows and 48 + 48 columns); key 2 = 1: the direct 3x3 kernels' 8-row tiles run as 8
 * waves of one row each (512 threads) instead of 4 waves of two rows; key 3 = 1: the
 * 18 / 36 / 72-channel 3x3 weight gradients spread their column tiles over 8 waves;
 * key 4 = the persistent 1x1 GEMM's maximum N tiles (of 16 channels) per workgroup, 3..8
 * (default 4); key 5 = 1: its row tiles of 16 instead of 32 pixels; key 6 = 1: gather-GEMM
 * convs with 18 / 36 output channels as 16 + 2 / 32 + 4 (VALU remainder columns); keys
 * 7-13: see vae2_conv2d_set_tune in csrc/conv.hip; key 14 = 1: the 72-channel direct 3x3
 * as two N blocks of 32 + 4 (off: measured slower); key 15 = 1 (default): direct 3x3
 * layers whose 4-row tiles leave <= 2 workgroups per CU split K over 8-wave workgroups
 * (2 = over 16-wave workgroups, 4 shares; 0 = off);
 * key 16 = the narrow 3x3 weight gradient's minimum tiles per partial slab (1..2, default 2);
 * key 17 = the streaming 3x3's minimum 4-row steps per band (1..2, default 1); key 18 = the
 * gather weight gradient's target workgroups (256..8192, default 1024); key 19 = BatchNorm
 * blocks per layer at most (256..8192, default 1024); key 20 = the multi-layer BatchNorm
 * apply kernels' resident-block budget (0 = one workgroup per pixel chunk, the default; R > 0:
 * ceil(T / ceil(T / R)) workgroups stride over the T chunks); key 21 = 0: the fuse sum +
 * ReLU one channel per thread instead of one channel quad (default 1).  Returns the previous value, -1 for an unknown key or an
 * out-of-range value of keys 4, 6, 7 and 15-20 (the setting is then left unchanged).    */
int vae2_conv2d_set_tune(int key, int value);
/* Deferred weight-gradient reductions: while on (a per-thread switch), every
 * vae2_conv2d_bwd_weight(_ld) launches its partial-slab kernel and queues the slab
 * reduction (one process-wide queue); vae2_wgrad_flush launches the queued reductions
 * together on `stream` (up to 32 per launch, in queue order; reductions into the same
 * dW elements go to successive launches).  The caller orders `stream` after the
 * streams the weight gradients were issued on and keeps each call's workspace alive
 * until the flush is enqueued.  Returns the previous setting.                        */
int vae2_wgrad_defer(int on);
int vae2_wgrad_flush(void* stream);
/* ABI 10: launch only the queued reductions that were queued from `stream`, on it (no
 * cross-stream ordering needed: a sub-network on a side stream -- the posterior net --
 * finishes its own weight gradients while other streams' stay queued).              */
int vae2_wgrad_flush_stream(void* stream);

/* Independent convolutions in one call (the lock-stepped layers of one HRNet depth
 * level).  Each job is one vae2_conv2d_fwd (kind 0: x, xd -> y, yd with bias, beta,
 * stats) or vae2_conv2d_bwd_data (kind 1: x, xd = dy -> y, yd = dx with beta; bias and
 * stats ignored) call with the same meaning; jobs the LDS-tiled direct 3x3 kernel
 * takes share launches (up to 4 per launch, grouped by tile shape; jobs writing the
 * same output never share one), the others are issued one by one.  The jobs must be
 * independent (no job reads another's output).  Grouping is off by default (measured
 * slower in the full training step, where side-stream concurrency already fills the
 * chip); vae2_conv2d_set_grouping(1) enables it; returns the previous setting.       */
typedef struct vae2_conv_job {
  int32_t kind, k, stride, pad;
  const float* x;
  vae2_act xd;
  const float* wp;
  const float* bias;
  float* y;
  vae2_act yd;
  float beta;
  float* stats;
} vae2_conv_job;
int vae2_conv2d_multi(int n, const vae2_conv_job* jobs, void* stream);
int vae2_conv2d_set_grouping(int on);

/* Conv weights are consumed in a packed layout (zero-padded, K = (tap, 4-channel
 * quad) ordered): mode 0 for vae2_conv2d_fwd  = [round_up(Cout,64)][k*k][round_up(Cin,4)],
 * mode 1 for vae2_conv2d_bwd_data = [round_up(Cin,64)][k*k][round_up(Cout,4)].
 * Size in floats / packing from the reference [Cout][Cin][k][k] layout:          */
int64_t vae2_conv2d_packed_size(int64_t cout, int64_t cin, int k, int mode);
int vae2_conv2d_pack_weight(const float* w, int64_t cout, int64_t cin, int k,
                            int mode, float* out, void* stream);
/* The same from a block of input channels of a wider weight: element (co, ci, t)
 * is read at w[co*ld + ci*k*k + t] (ld >= cin*k*k; pass w + c0*k*k for the block
 * starting at input channel c0).                                                */
int vae2_conv2d_pack_weight_ld(const float* w, int64_t cout, int64_t cin, int k,
                               int mode, int64_t ld, float* out, void* stream);

/* Many packings in one launch (a model's whole weight set after each optimizer
 * step).  `jobs` is a DEVICE array of njobs descriptors; `out` buffers must not
 * overlap.  Replaces the per-conv weight reads of F.conv2d (enc_hrnet.py:27-30). */
typedef struct vae2_pack_job {
  const float* w;  /* [cout][cin][k][k], rows ld floats apart */
  float* out;      /* vae2_conv2d_packed_size(cout, cin, k, mode) floats */
  int32_t cout, cin, k, mode;
  int32_t ld;      /* 0: cin*k*k (a whole weight), else as vae2_conv2d_pack_weight_ld */
  int32_t pad_;
} vae2_pack_job;
int vae2_conv2d_pack_weights(const vae2_pack_job* jobs, int64_t njobs, void* stream);

/* y = conv2d(x, w, stride, pad) (+ bias) (+ beta*y) with w packed (mode 0),
 * optional per-channel BN partial sums of the result in `stats` ([2][rows][cout]).
 * Replaces nn.Conv2d.forward: conv3x3 enc_hrnet.py:27-30, Bottleneck 1x1
 * :70-76, downsample :411-415, fuse :188-217, transitions :381-403, heads
 * :323-370/:598-750, z head :1026-1039.                                       */
int vae2_conv2d_fwd(const float* x, const vae2_act* xd, const float* wp,
                    const float* bias, float* y, const vae2_act* yd, int k,
                    int stride, int pad, float beta, float* stats,
                    void* stream);

/* BatchNorm fused into the consumer conv (ABI 9).  A conv2d whose input is the
 * normalised output relu?(x*scale + shift) of a training-mode BatchNorm (+ReLU) layer
 * (BasicBlock's bn1 -> relu -> conv2, enc_hrnet.py:46-55) can read that layer's pre-BN
 * tensor x and its save [4][C] = (mean, invstd, scale, shift) instead, so the normalised
 * activation is never stored: _fwd_bnin / _bwd_weight_bnin are vae2_conv2d_fwd /
 * vae2_conv2d_bwd_weight of that input (bit-identical to normalising first), legal when
 * vae2_conv2d_bnin_ok (the LDS-tiled direct 3x3 kernels run).  Its data gradient can
 * also produce the BatchNorm layer's backward partials [2][rows][C] (sum g, sum g*xhat
 * with g the incoming gradient masked by the ReLU, as vae2_bn_relu_bwd_reduce writes)
 * in the epilogue: rows = vae2_conv2d_bwd_data_bnpart_rows (0 = not available for
 * this geometry); bn_x = the BatchNorm's pre-BN input (shape of dx).  Since round 6
 * (same ABI) every data-gradient kernel family writes them -- the direct 3x3 kernels,
 * the persistent 1x1 GEMM and the gather kernel (1x1, 3x3, stride-2 parity classes) --
 * so any conv that is the ONLY consumer of a stored BatchNorm(+ReLU) output without
 * residual can replace that layer's backward reduce pass (vae2/ops.py PartBN).      */
int vae2_conv2d_bnin_ok(const float* x, const vae2_act* xd, const vae2_act* yd, int k,
                        int stride, int pad);
int vae2_conv2d_fwd_bnin(const float* x, const vae2_act* xd, const float* bn_save, int relu,
                         const float* wp, const float* bias, float* y, const vae2_act* yd,
                         int k, int stride, int pad, float beta, float* stats, void* stream);
int vae2_conv2d_bwd_weight_bnin(const float* x, const vae2_act* xd, const float* bn_save,
                                int relu, const float* dy, const vae2_act* dyd, float* dw,
                                float* dbias, int k, int stride, int pad, int accumulate,
                                float* ws, int64_t ws_size, void* stream);
int64_t vae2_conv2d_bwd_data_bnpart_rows(const float* dy, const vae2_act* dyd,
                                         const vae2_act* dxd, int k, int stride, int pad);
int vae2_conv2d_bwd_data_bnpart(const float* dy, const vae2_act* dyd, const float* wp,
                                float* dx, const vae2_act* dxd, int k, int stride, int pad,
                                const float* bn_x, const vae2_act* bn_xd, const float* bn_save,
                                int relu, float* partials, void* stream);

/* Name of the kernel instantiation a vae2_conv2d_fwd launch with this geometry
 * uses (e.g. "igemm_kernel<4, 4, true, 0>"), for matching timings with rocprof. */
int vae2_conv2d_fwd_kernel_name(const vae2_act* xd, const vae2_act* yd, int k, int stride,
                                int pad, char* buf, int64_t len);

/* dx = conv2d_transpose(dy, w) (+ beta*dx) with w packed (mode 1): gradient of
 * vae2_conv2d_fwd w.r.t. its input (autograd's convolution_backward, input half). */
int vae2_conv2d_bwd_data(const float* dy, const vae2_act* dyd, const float* wp,
                         float* dx, const vae2_act* dxd, int k, int stride,
                         int pad, float beta, void* stream);

/* Workspace (floats) needed by vae2_conv2d_bwd_weight for this shape.         */
int64_t vae2_conv2d_bwd_weight_ws_size(const vae2_act* xd, const vae2_act* dyd,
                                       int k);

/* dw (+)= sum_pixels dy (x) im2col(x); dbias (+)= sum_pixels dy if dbias.
 * accumulate != 0 adds into dw/dbias (gradient buffers), else overwrites.
 * (autograd's convolution_backward, weight half.)                            */
int vae2_conv2d_bwd_weight(const float* x, const vae2_act* xd, const float* dy,
                           const vae2_act* dyd, float* dw, float* dbias, int k,
                           int stride, int pad, int accumulate, float* ws,
                           int64_t ws_size, void* stream);

/* vae2_conv2d_bwd_weight writing dW rows dw_ld floats apart (an input-channel
 * block of a wider weight's gradient: dw = grad + c0*k*k, dw_ld = Cin_total*k*k). */
int vae2_conv2d_bwd_weight_ld(const float* x, const vae2_act* xd, const float* dy,
                              const vae2_act* dyd, float* dw, int64_t dw_ld, float* dbias,
                              int k, int stride, int pad, int accumulate, float* ws,
                              int64_t ws_size, void* stream);

/* ------------------------------------------------------------ batchnorm ---- */
/* nn.BatchNorm2d(momentum=0.01, eps=1e-5) in train mode, enc_hrnet.py:22-23,
 * (SyncBatchNorm when distributed, tools/train.py:216-218).                   */

/* Rows of partials written by vae2_bn_stats / vae2_bn_relu_bwd_reduce.        */
int64_t vae2_bn_partial_rows(const vae2_act* xd);

/* Per-channel partial sums of x and x^2 -> partials [2][rows][c].             */
int vae2_bn_stats(const float* x, const vae2_act* xd, float* partials,
                  void* stream);

/* partials [2][rows][c] (float) -> sums [2][c] (double, summed in fixed order).
 * With accumulate != 0 the result is added to `sums`.                         */
int vae2_bn_partials_reduce(const float* partials, int64_t rows, int64_t c,
                            double* sums, int accumulate, void* stream);

/* sums [2][c] = (sum x, sum x^2) over `count` values per channel (after an
 * optional cross-rank all-reduce) -> save [4][c] = (mean, invstd, scale, shift)
 * with scale = gamma*invstd, shift = beta - mean*scale; updates running stats
 * (unbiased variance) and num_batches_tracked when those pointers are set.   */
int vae2_bn_finalize(const double* sums, double count, const float* gamma,
                     const float* beta, float* running_mean, float* running_var,
                     int64_t* num_batches_tracked, float momentum, float eps,
                     int64_t c, float* save, void* stream);

/* vae2_bn_partials_reduce + vae2_bn_finalize in one launch (no cross-rank
 * exchange in between: single GPU, or BN without SyncBN).                      */
int vae2_bn_reduce_finalize(const float* partials, int64_t rows, int64_t c,
                            double* sums, double count, const float* gamma,
                            const float* beta, float* running_mean, float* running_var,
                            int64_t* num_batches_tracked, float momentum, float eps,
                            float* save, void* stream);

/* The same with shifted statistics: partials / sums hold sums of (x - mean_shift[c])
 * (vae2_conv1x1_upsum_fwd's, centred on the conv bias so E[x^2] - E[x]^2 does not
 * cancel); the mean (save, running_mean) gets mean_shift back.  mean_shift may be NULL. */
int vae2_bn_reduce_finalize_shifted(const float* partials, int64_t rows, int64_t c,
                                    double* sums, double count, const float* mean_shift,
                                    const float* gamma, const float* beta,
                                    float* running_mean, float* running_var,
                                    int64_t* num_batches_tracked, float momentum, float eps,
                                    float* save, void* stream);
int vae2_bn_finalize_shifted(const double* sums, double count, const float* mean_shift,
                             const float* gamma, const float* beta, float* running_mean,
                             float* running_var, int64_t* num_batches_tracked, float momentum,
                             float eps, int64_t c, float* save, void* stream);

/* Backward: partials [2][rows][c] of (sum g, sum g*xhat) -> sums [2][c] (double)
 * and dgamma += sum g*xhat, dbeta += sum g, in one launch.                       */
int vae2_bn_bwd_reduce_param_grads(const float* partials, int64_t rows, int64_t c,
                                   double* sums, float* dgamma, float* dbeta,
                                   void* stream);

/* Eval mode: save [4][c] from running statistics.                              */
int vae2_bn_eval_coeffs(const float* gamma, const float* beta,
                        const float* running_mean, const float* running_var,
                        float eps, int64_t c, float* save, void* stream);

/* y = fma(x, scale, shift) (+ res) (then ReLU if relu).  Only channels [0, c)
 * of each pixel are written.                                                  */
int vae2_bn_apply(const float* x, const vae2_act* xd, const float* save,
                  const float* res, const vae2_act* rd, float* y,
                  const vae2_act* yd, int relu, void* stream);

/* Backward reduce: g = dy * (y > 0 if relu); partials [2][rows][c] of
 * (sum g, sum g*xhat), xhat = (x - mean)*invstd.  With relu and y == NULL the
 * mask is recomputed as fma(x, scale, shift) > 0 — exactly vae2_bn_apply's
 * forward output when it had no residual — saving the read of y.              */
int vae2_bn_relu_bwd_reduce(const float* dy, const vae2_act* dyd,
                            const float* y, const vae2_act* yd, const float* x,
                            const vae2_act* xd, const float* save, int relu,
                            float* partials, void* stream);

/* dgamma (+)= sum g*xhat, dbeta (+)= sum g from local sums [2][c].            */
int vae2_bn_bwd_param_grads(const double* sums, int64_t c, float* dgamma,
                            float* dbeta, void* stream);

/* dx = gamma*invstd*(g - sum_g/count - xhat*sum_gxhat/count);
 * also dres = g when dres != NULL (residual branch of the block).  The ReLU
 * mask comes from y, or from x as in vae2_bn_relu_bwd_reduce when y == NULL. */
int vae2_bn_relu_bwd_apply(const float* dy, const vae2_act* dyd, const float* y,
                           const vae2_act* yd, const float* x,
                           const vae2_act* xd, const float* save,
                           const float* gamma, const double* sums, double count,
                           int relu, float* dx, const vae2_act* dxd,
                           float* dres, const vae2_act* dresd, void* stream);

/* Multi-layer BatchNorm launches: the independent BN layers of one HRNet depth level
 * (a HighResolutionModule's branches run in lockstep, its fuse convs, transition
 * units) share each launch instead of one launch per layer (~3x fewer BN launches),
 * and with SyncBN their statistics cross ranks in one exchange.  Same math as the
 * single-layer calls above.  Layer tensors: 16-byte aligned NHWC, pixel stride % 4
 * == 0, C <= 1024.  Any n (split into launches of 6 layers).                       */
typedef struct vae2_bn_layer {
  const float* x; vae2_act xd;    /* pre-BN activation (the conv output)               */
  const float* a; vae2_act ad;    /* forward: residual, backward: y for the ReLU mask;  */
                                  /* NULL: none / mask recomputed from x               */
  float* o; vae2_act od;          /* forward: y; backward: dx                          */
  const float* dy; vae2_act dyd;  /* backward                                          */
  float* dres; vae2_act dresd;    /* backward: residual gradient (= masked dy) or NULL  */
  const float* save;              /* [4][c]: mean, invstd, scale, shift                 */
  const float* gamma;             /* backward apply (NULL: 1)                            */
  float* partials;                /* backward reduce: [2][vae2_bn_partial_rows(xd)][c]  */
  const double* sums;             /* backward apply: (sum g, sum g*xhat) [2][c]         */
  const double* countp;           /* device element count per channel (SyncBN: summed  */
  double count;                   /* over ranks), or NULL to use `count`               */
  int relu;
  int dres_acc;                   /* backward apply: 1 = dres += masked dy (the residual  */
                                  /* gradient summed onto another consumer's, in-kernel) */
  /* ABI 10: the residual through its own BatchNorm (no ReLU) whose normalised output is
   * never stored -- the Bottleneck's downsample shortcut (enc_hrnet.py:94-101, replaces
   * a separate apply pass, backward reduce pass and backward apply pass of that BN).
   * rx = NULL: none.  Forward (a must be NULL): y = relu?(fma(x, scale, shift) +
   * fma(rx, rsave.scale, rsave.shift)).  Backward (dres must be NULL): the residual BN's
   * partials (sum g, sum g*xhat_r) into rpartials (reduce) and its input gradient
   * rgamma*rinvstd*(g - rsums_g/count - xhat_r*rsums_gx/count) into rdx (apply), g =
   * this layer's masked dy.  Same pixels and channels as x.                            */
  const float* rx; vae2_act rxd;
  const float* rsave;             /* [4][c] of the residual BN                          */
  const float* rgamma;            /* backward apply (NULL: 1)                            */
  float* rpartials;               /* backward reduce: [2][vae2_bn_partial_rows(xd)][c]  */
  const double* rsums;            /* backward apply: the residual BN's [2][c] sums       */
  float* rdx; vae2_act rdxd;      /* backward apply: the residual BN's input gradient   */
  /* ABI 10: the ReLU mask as one byte per (pixel, channel quad), bit k = (y[4q+k] > 0),
   * [P][ceil(c/4)]: written by vae2_bn_multi_apply when non-NULL, read by the backward
   * passes instead of y (a) -- 1/16 of y's bytes.  NULL: y / recomputed from x.         */
  unsigned char* mask;
} vae2_bn_layer;
/* y = relu?(fma(x, scale, shift) + a) per layer (vae2_bn_apply).                 */
int vae2_bn_multi_apply(int n, const vae2_bn_layer* layers, void* stream);
/* partials of (sum g, sum g*xhat) per layer (vae2_bn_relu_bwd_reduce).            */
int vae2_bn_multi_bwd_reduce(int n, const vae2_bn_layer* layers, void* stream);
/* dx (and dres) per layer (vae2_bn_relu_bwd_apply).                              */
int vae2_bn_multi_bwd_apply(int n, const vae2_bn_layer* layers, void* stream);

typedef struct vae2_bn_fin {
  const float* partials; int64_t rows; int64_t c;  /* [2][rows][c] fp32 partial rows   */
  double* sums;                   /* [2][c] out (mode 2 / finalize: in)                 */
  const double* countp;           /* device count, or NULL to use `count`               */
  double count;
  const float* gamma; const float* beta;
  float* running_mean; float* running_var; int64_t* num_batches_tracked;  /* or NULL  */
  float momentum, eps;
  float* save;                    /* [4][c] out (mode 0 / finalize)                     */
  float* dgamma; float* dbeta;    /* mode 1: += (sum g*xhat, sum g), or NULL            */
} vae2_bn_fin;
/* Per layer, partial rows -> sums in double (fixed order), then mode 0: finalize
 * (save + running statistics, vae2_bn_reduce_finalize), mode 1: backward parameter
 * gradients (vae2_bn_bwd_reduce_param_grads), mode 2: sums only (SyncBN: exchange,
 * then vae2_bn_multi_finalize).                                                    */
int vae2_bn_multi_reduce(int n, const vae2_bn_fin* fins, int mode, void* stream);
/* save + running statistics from sums (vae2_bn_finalize).                         */
int vae2_bn_multi_finalize(int n, const vae2_bn_fin* fins, void* stream);

/* ---------------------------------------------------------- head output ---- */
/* 1x1 conv of a channel-concatenation of bilinearly upsampled maps, computed per
 * block of input channels (the HRNet heads, enc_hrnet.py:833-847, :889-905, :947-963:
 * Conv1x1(cat[x0, up(x1), up(x2), up(x3)])).  A 1x1 conv commutes with the
 * upsampling, so with W = [W0 | W1 | W2 | W3] split by input block
 *     y = W0 x0 + bias + up(W1 x1) + up(W2 x2) + up(W3 x3),
 * the z_s = W_s x_s computed at their own resolution (vae2_conv2d_fwd).  This call:
 * y = conv1x1(x, wp) + bias + sum_s bilinear_up(ups[s]) to y's h, w (align_corners=False;
 * channels [0, yd->c) of each ups[s], nup <= 3), wp = the W0 block packed as
 * vae2_conv2d_pack_weight(_ld) mode 0 (Cin0 <= 32); optional BN partial statistics
 * stats [2][vae2_conv1x1_upsum_stats_rows(yd)][Cout] of y - bias (shifted: finalize
 * with vae2_bn_reduce_finalize_shifted / vae2_bn_finalize_shifted, mean_shift = bias).
 * y is written in the 64-channel-blocked layout B64 (not NHWC):
 *     element (p, c) at y[(c / 64) * P * 64 + p * 64 + c % 64],  P = n*h*w,
 * i.e. ceil(Cout/64) * P * 64 floats (yd->ps is ignored).                          */
int64_t vae2_conv1x1_upsum_stats_rows(const vae2_act* yd);
int vae2_conv1x1_upsum_fwd(const float* x, const vae2_act* xd, const float* wp,
                           const float* bias, int nup, const float* const* ups,
                           const vae2_act* upds, float* y, const vae2_act* yd, float* stats,
                           void* stream);

/* The HRNet head after its wide 1x1 conv (enc_hrnet.py:323-370, applied at
 * :839-847, :897-905, :955-963): BatchNorm (coefficients `save` [4][C] from
 * vae2_bn_reduce_finalize / _finalize) -> ReLU -> Conv1x1(C -> cout2 <= 4, bias),
 * reading the pre-BN conv output y once per pass; the ReLU output is never stored.
 * y: the B64 layout of vae2_conv1x1_upsum_fwd, 16-byte aligned, C <= 1024 (dy: NHWC).  w2 = [cout2][C] (the conv weight
 * [cout2][C][1][1]), b2 = [cout2] or NULL.
 *   out[p][o] = b2[o] + sum_c w2[o][c] * relu(y[p][c]*scale[c] + shift[c])        */
int vae2_head_out_fwd(const float* y, const vae2_act* yd, const float* save, const float* w2,
                      const float* b2, int cout2, float* out, const vae2_act* outd,
                      void* stream);
/* Workspace (floats) of the two backward calls.                                   */
int64_t vae2_head_out_bwd_ws_size(const vae2_act* yd, int cout2);
/* Backward, part 1 (local sums; SyncBN all-reduces `sums` before part 2):
 * g = (w2^T dout) * [relu input > 0];  sums[2][C] = (sum g, sum g*xhat) in double;
 * dgamma += sum g*xhat, dbeta += sum g, dw2 += sum dout (x) relu_out, db2 += sum dout
 * (any of the four may be NULL).                                                   */
int vae2_head_out_bwd_reduce(const float* y, const vae2_act* yd, const float* save,
                             const float* w2, int cout2, const float* dout,
                             const vae2_act* doutd, double* sums, float* dgamma, float* dbeta,
                             float* dw2, float* db2, float* ws, int64_t ws_size, void* stream);
/* Backward, part 2: dy = gamma*invstd*(g - sums[0]/count - xhat*sums[1]/count) (the
 * gradient w.r.t. the wide conv's output), dbias += sum_p dy when dbias != NULL.     */
int vae2_head_out_bwd_apply(const float* y, const vae2_act* yd, const float* save,
                            const float* gamma, const float* w2, int cout2, const float* dout,
                            const vae2_act* doutd, const double* sums, double count, float* dy,
                            const vae2_act* dyd, float* dbias, float* ws, int64_t ws_size,
                            void* stream);

/* ----------------------------------------------- resample / fuse / concat ---- */

/* y (+)= bilinear_upsample(x) to y's h,w, align_corners=False
 * (F.interpolate/F.upsample mode='bilinear', enc_hrnet.py:242-245, :835-837,
 * :1111-1113). beta: y = up(x) + beta*y.                                      */
int vae2_upsample_bilinear_fwd(const float* x, const vae2_act* xd, float* y,
                               const vae2_act* yd, float beta, void* stream);
/* dx (+)= adjoint of the above applied to dy (beta: dx = adj + beta*dx).      */
int vae2_upsample_bilinear_bwd(const float* dy, const vae2_act* dyd, float* dx,
                               const vae2_act* dxd, float beta, void* stream);

/* y = relu(sum_i up(x_i)) over n <= 4 terms; terms with smaller h,w than y
 * are bilinearly upsampled (HighResolutionModule fuse, enc_hrnet.py:233-249). */
int vae2_fuse_sum_relu(int n, const float* const* xs, const vae2_act* xds,
                       float* y, const vae2_act* yd, void* stream);
/* ABI 10: as vae2_fuse_sum_relu, with saves[i] (or NULL) the BatchNorm [4][c] (mean,
 * invstd, scale, shift) of term i: x_i is then that BN's pre-BN input r and the term is
 * fma(r, scale, shift) (the fuse unit's BN output, enc_hrnet.py:199-218, never stored). */
int vae2_fuse_sum_relu_bn(int n, const float* const* xs, const vae2_act* xds,
                          const float* const* saves, float* y, const vae2_act* yd,
                          void* stream);

/* Head-kernel variants (A/B measurement): bit 0 = the per-channel-lane vertical pass of
 * the power-of-two upsampling adjoint instead of the row-streaming one; bit 1 = the
 * up-sum kernel with 12 staging columns for every source (instead of 12 / 6 / 3 for
 * halving source resolutions); bit 2 = the two-pass (horizontal, then vertical through a
 * workspace) power-of-two adjoint instead of the one-pass band kernel; bit 3 = the
 * LDS-staged up-sum instead of the one-pass kernel; bits 4 / 5 = 4 instead of 2 pixels in
 * flight per thread in the head backward reduce / apply passes; bit 6 = the fuse layers'
 * pow2 adjoints through the one-pass band kernel (off by default); bit 7 = the scalar
 * ReLU-backward (dual)
 * kernel instead of the channel-quad one; bits 8-15 = the
 * one-pass kernel's dy rows per workgroup (a multiple of 8; 0 = 32).  Returns the
 * previous setting.  Process-wide.                                                    */
int vae2_heads_set_algo(int algo);

/* dxs[s] = adjoint of bilinear_up (align_corners=False) applied to dy, for n <= 3
 * lower-resolution targets at once, reading dy once (separable: a horizontal pass into
 * the workspace, then a vertical pass per target).  dxs[s] have dy's channel count.  */
int64_t vae2_upsample_bilinear_bwd_multi_ws_size(const vae2_act* dyd, int n,
                                                 const vae2_act* dxds);
int vae2_upsample_bilinear_bwd_multi(const float* dy, const vae2_act* dyd, int n,
                                     float* const* dxs, const vae2_act* dxds, float* ws,
                                     int64_t ws_size, void* stream);

/* dxs[s] = adj(dy) + betas[s]*dxs[s] (betas may be NULL: 0) for n <= 3 targets whose h
 * and w are dy's divided by the same 2, 4 or 8 (any order): the HighResolutionModule
 * fuse backward (enc_hrnet.py:233-249, the lower branches' upsample terms of one output
 * row), thread per (pixel, channel quad) for narrow channel counts.  _ws_size returns
 * the workspace in floats, or -1 when a target is not such a downsampling (callers
 * then take vae2_upsample_bilinear_bwd per target).  dy and ws 16-byte aligned,
 * dyd->ps % 4 == 0.                                                             */
int64_t vae2_upsample_bilinear_bwd_pow2_ws_size(const vae2_act* dyd, int n,
                                                const vae2_act* dxds);
int vae2_upsample_bilinear_bwd_pow2(const float* dy, const vae2_act* dyd, int n,
                                    float* const* dxs, const vae2_act* dxds,
                                    const float* betas, float* ws, int64_t ws_size,
                                    void* stream);

/* g = dy * (y > 0)  (ReLU backward, threshold_backward).                       */
int vae2_relu_bwd(const float* dy, const vae2_act* dyd, const float* y,
                  const vae2_act* yd, float* g, const vae2_act* gd,
                  void* stream);

/* g = dy * (y > 0) and g2 = g + beta2 * g2 in one pass: the ReLU gradient of an HRNet
 * fuse output handed both to its own consumers and, accumulated, to the shared
 * gradient buffer of a branch input with several consumers (vae2/ops.py GradLink).  */
int vae2_relu_bwd_dual(const float* dy, const vae2_act* dyd, const float* y,
                       const vae2_act* yd, float* g, const vae2_act* gd, float* g2,
                       const vae2_act* g2d, float beta2, void* stream);

/* y = x (strided NHWC copy, e.g. into a channel slice for torch.cat).         */
int vae2_copy_act(const float* x, const vae2_act* xd, float* y,
                  const vae2_act* yd, float beta, void* stream);

/* Code-map tiling (_gen_code_map, enc_hrnet.py:454-462): y[n,:,:,c] = v[n,c]
 * for a per-clip vector v [n][vc] (vector stride vs).                          */
int vae2_codemap_tile_fwd(const float* v, int64_t vs, float* y,
                          const vae2_act* yd, void* stream);
/* Workspace (floats) for the spatial reductions below.                          */
int64_t vae2_spatial_ws_size(const vae2_act* xd);
/* dv (+)= sum over h,w of dy[n,:,:,c].                                          */
int vae2_codemap_tile_bwd(const float* dy, const vae2_act* dyd, float* dv,
                          int64_t vs, int accumulate, float* ws, int64_t ws_size,
                          void* stream);

/* NCHW <-> NHWC layout conversion at the API boundary (clips are (B, 3L, H, W)
 * tensors, cityscapes.py:311-326).                                             */
int vae2_nchw_to_nhwc(const float* x, float* y, const vae2_act* yd,
                      float beta, void* stream);
int vae2_nhwc_to_nchw(const float* x, const vae2_act* xd, float* y,
                      float beta, void* stream);

/* AdaptiveAvgPool2d((1,1)) (enc_hrnet.py:1025): y[n][c] = mean_hw x.           */
int vae2_global_avgpool_fwd(const float* x, const vae2_act* xd, float* y,
                            const vae2_act* yd, float* ws, int64_t ws_size,
                            void* stream);
int vae2_global_avgpool_bwd(const float* dy, const vae2_act* dyd, float* dx,
                            const vae2_act* dxd, float beta, void* stream);
/* AdaptiveAvgPool2d((1,1)) of F.upsample(x, (H, W), bilinear) (enc_hrnet.py:1022-1025,
 * the posterior net's pooled concat) without the full-resolution tensor: the mean of a
 * bilinear upsampling is a separably weighted sum at the source resolution,
 * y[n][c] = scale * sum_{iy,ix} x[n][iy][ix][c] * wr[iy] * wc[ix]  (wr / wc: device
 * [h] / [w] column sums of the interpolation weights, scale = 1 / (H*W)); ws:
 * vae2_spatial_ws_size(xd) floats.  The backward is the weighted broadcast
 * dx (+)= scale * dy[n][c] * wr[iy] * wc[ix]  (beta 0: overwrite, 1: accumulate).       */
int vae2_weighted_avgpool_fwd(const float* x, const vae2_act* xd, const float* wr,
                              const float* wc, float scale, float* y, const vae2_act* yd,
                              float* ws, int64_t ws_size, void* stream);
int vae2_weighted_avgpool_bwd(const float* dy, const vae2_act* dyd, const float* wr,
                              const float* wc, float scale, float* dx, const vae2_act* dxd,
                              float beta, void* stream);

/* ------------------------------------------------------------- ELBO ---- */

/* out[0] = sum |p - t| * scale  (L1Loss, criterion.py:61-69, scale = 1/B).
 * ws: vae2_reduce_ws_size(n elements) floats.                                  */
int64_t vae2_reduce_ws_size(int64_t n);
int vae2_l1_fwd(const float* p, const vae2_act* pd, const float* t,
                const vae2_act* td, float scale, float* ws, float* out,
                void* stream);
/* dp (+)= sign(p - t) * scale * gout[0] * (beta ? +prev : )                   */
int vae2_l1_bwd(const float* p, const vae2_act* pd, const float* t,
                const vae2_act* td, const float* gout, float scale, float* dp,
                const vae2_act* dpd, float beta, void* stream);

/* LSGAN term (criterion.py:90-103: MSELoss(reduction='sum') against ones for 'real',
 * zeros for 'fake', divided by the batch): out[0] = scale * sum (x - target)^2,
 * target = 1 or 0, scale = 1/B (x 0.5 at the call sites, utils.py:114-119, :256-266).
 * ws: vae2_reduce_ws_size(elements) floats.                                     */
int vae2_lsgan_fwd(const float* x, const vae2_act* xd, float target, float scale, float* ws,
                   float* out, void* stream);
/* dx (+)= 2 * scale * gout[0] * (x - target)   (beta 0: overwrite, 1: accumulate)  */
int vae2_lsgan_bwd(const float* x, const vae2_act* xd, float target, const float* gout,
                   float scale, float* dx, const vae2_act* dxd, float beta, void* stream);

/* Reparameterisation + KL (utils.py:85-101, criterion.py:72-87).
 * muvar: act with 2*zc channels (mu = [0,zc), logvar = [zc,2zc)); eps, z: acts
 * with zc channels.  prior != 0: z = eps (prior_sampling).
 * kl_out[0] (+)= scale * sum 0.5*(mu^2 + exp(lv) - lv - 1).                     */
int vae2_reparam_kl_fwd(const float* muvar, const vae2_act* md,
                        const float* eps, const vae2_act* ed, float* z,
                        const vae2_act* zd, int prior, float scale,
                        float* kl_out, int accumulate, float* ws, void* stream);
/* dmuvar = dz-path + gkl[0]*scale*dKL;  dz may be NULL (no z gradient).        */
int vae2_reparam_kl_bwd(const float* muvar, const vae2_act* md,
                        const float* eps, const vae2_act* ed, const float* dz,
                        const vae2_act* dzd, const float* gkl, float scale,
                        float* dmuvar, const vae2_act* dmd, void* stream);

/* total[0] = sum_i lambda_i * terms[i][0] (utils.py:150-152); n <= 8.          */
int vae2_weighted_sum(int n, const float* const* terms, const float* lambdas,
                      float* total, void* stream);

/* flag[0] |= any(!isfinite(x)) (FullModel_encdec._anomoly_detection,
 * utils.py:63-65). x is a dense array of n floats.                              */
int vae2_nonfinite_check(const float* x, int64_t n, int32_t* flag,
                         void* stream);

/* ------------------------------------------------------------ clip input ---- */

/* CityscapesSequence.input_transform + __getitem__ (cityscapes.py:311-326): a batch of
 * uint8 RGB frame windows frames[n][nframes][h][w][3] (dense, 4-byte aligned) becomes
 * nseg NCHW fp32 segment tensors outs[s][n][3*nframes/nseg][h][w], channel 3*f + rgb,
 * value lut[rgb*256 + byte].  The caller tabulates the reference's per-element
 * arithmetic ((byte/255 in fp32 - mean) / std in fp64, rounded to fp32: vae2/clips.py
 * normalize_lut) as a [3][256] fp32 device table.  nseg in [1, 8], nseg | nframes.   */
int vae2_clip_normalize_u8(const uint8_t* frames, int64_t n, int64_t nframes, int64_t h,
                           int64_t w, const float* lut, int nseg, float* const* outs,
                           void* stream);

/* --------------------------------------------------------- eval metrics ---- */

/* _to_image (function.py:86-97) over NCHW fp32 planes, RGB = channel % 3:
 * y = clip((fp32(fp32(x * std) + mean)) * 255, 0, 255) (x*std and +mean in fp64 as
 * numpy does for a float32 array against the fp64 mean/std arrays).  mean3 / std3 are
 * HOST arrays.  y may alias x.                                                    */
int vae2_to_image(const float* x, float* y, int64_t n, int64_t c, int64_t h, int64_t w,
                  const double* mean3, const double* std3, void* stream);
/* Workspace (doubles) for vae2_absdiff_sqdiff_sum / vae2_ssim over `planes` h x w
 * planes.                                                                         */
int64_t vae2_metrics_ws_size(int64_t planes, int64_t h, int64_t w);
/* out[0] = sum |a - b|, out[1] = sum (a - b)^2 over n floats, in double (device out):
 * the recon_loss (function.py:252) and PSNR (criterion.py:106-116) sums.          */
int vae2_absdiff_sqdiff_sum(const float* a, const float* b, int64_t n, double* ws,
                            double* out, void* stream);
/* pytorch_msssim _ssim (restated from pytorch_msssim 1.0.0, used at function.py:244-251):
 * per plane p of x, y ([planes][h][w] fp32, h, w >= 11): the 11-tap separable window
 * `win` (valid filtering) gives mu, sigma; out[2p] = mean SSIM map, out[2p+1] = mean
 * contrast-structure map, C1 = (K1*L)^2, C2 = (K2*L)^2.  Device out, double.       */
int vae2_ssim(const float* x, const float* y, int64_t planes, int64_t h, int64_t w,
              const float* win, int win_size, float c1, float c2, double* ws, double* out,
              void* stream);
/* F.avg_pool2d(kernel 2, stride 2, padding (h % 2, w % 2)) of each plane (the MS-SSIM
 * level step): y is [planes][(h + 2*(h%2) - 2)/2 + 1][(w + 2*(w%2) - 2)/2 + 1].     */
int vae2_avgpool2x2(const float* x, float* y, int64_t planes, int64_t h, int64_t w,
                    void* stream);

/* ------------------------------------------------------------ optimizer ---- */

/* torch.optim.Adam step (tools/train.py:251-261) over one flat fp32 buffer:
 * m = b1*m + (1-b1)*g ; v = b2*v + (1-b2)*g^2 ;
 * p -= lr/(1-b1^step) * m / (sqrt(v)/sqrt(1-b2^step) + eps)   (+ L2 wd).      */
int vae2_adam_step(float* p, const float* g, float* m, float* v, int64_t n,
                   float lr, float beta1, float beta2, float eps,
                   float weight_decay, int64_t step, void* stream);

/* The same step with the step counter and learning rate in device memory, so a
 * captured HIP graph can replay it: vae2_adam_coeffs increments state[0] (step,
 * double) and writes coeffs = {lr/(1-b1^step), sqrt(1-b2^step)} from lr = state[1];
 * vae2_adam_step_dev then updates each flat buffer from those coefficients.    */
int vae2_adam_coeffs(double* state, float beta1, float beta2, float* coeffs,
                     void* stream);
int vae2_adam_step_dev(float* p, const float* g, float* m, float* v, int64_t n,
                       const float* coeffs, float beta1, float beta2, float eps,
                       float weight_decay, void* stream);

/* dst = src * scale, for fp32 buffers (grad averaging after all-reduce).       */
int vae2_scale(float* dst, const float* src, int64_t n, float scale,
               void* stream);

/* ------------------------------------------------------ SyncBN exchange ---- */

/* ABI 11: one-shot peer all-reduce of the SyncBatchNorm statistics between the ranks of
 * one node (replaces the per-layer SyncBatchNorm all-reduces of the reference's DDP setup,
 * tools/train.py:216-218; vae2/dist.py makes one exchange per BN depth level).  Every rank
 * stores its payload into a slot of every rank's receive area (IPC-mapped device memory,
 * xGMI), raises its arrival flag there, waits for all flags of its own area and sums the
 * world payloads in rank order: identical doubles on every rank, one kernel per exchange.
 * Setup (collective): vae2_syncbn_comm_init allocates and zeroes this rank's area
 * (vae2_syncbn_comm_bytes) and writes its 64-byte IPC handle; the handles of all ranks,
 * concatenated in rank order, go to vae2_syncbn_comm_connect.  n <= max_elems doubles
 * per call; the calls are stream-ordered and must be made in the same order on every
 * rank (a HIP graph may capture them).  Waits are bounded (60 s by default,
 * vae2_syncbn_comm_set_timeout): a missing peer sets the error word (vae2_syncbn_comm_error,
 * a synchronous read) instead of hanging.  ABI 12: a failure is sticky and visible in the
 * data -- the timed-out exchange and every later one on this comm write NaN into buf and
 * exchange nothing (no payload, no flag), so the statistics turn NaN and the step's NaN/Inf
 * checks fire even where the error word is never read.  The receive areas are uncached
 * device memory.  world <= 8.                                                              */
typedef struct vae2_syncbn_comm vae2_syncbn_comm;
int64_t vae2_syncbn_comm_bytes(int world, int64_t max_elems);
int vae2_syncbn_comm_init(int rank, int world, int64_t max_elems, void* handle_out,
                          vae2_syncbn_comm** out);
int vae2_syncbn_comm_connect(vae2_syncbn_comm* comm, const void* handles);
int vae2_syncbn_allreduce(vae2_syncbn_comm* comm, double* buf, int64_t n, void* stream);
int vae2_syncbn_comm_error(vae2_syncbn_comm* comm, int64_t* host_out);
int vae2_syncbn_comm_set_timeout(vae2_syncbn_comm* comm, double seconds);
int vae2_syncbn_comm_destroy(vae2_syncbn_comm* comm);

#ifdef __cplusplus
}
#endif

#endif /* VAE2_HIP_H */
