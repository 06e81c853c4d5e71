// Training-mode BatchNorm2d (+ fused ReLU / residual) for NHWC fp32 activations.
//
// Replaces nn.BatchNorm2d(momentum=0.01, eps=1e-5) at enc_hrnet.py:22-23 and its
// autograd backward (native_batch_norm_backward) plus the ReLU / residual add of
// BasicBlock (:46-62) and Bottleneck (:83-103).
//
// Reductions are two-level and deterministic: a "partials" kernel writes one row
// of per-channel fp32 sums per block (fixed pixel ranges), then one block per
// channel sums the rows in double in a fixed tree order.  With SyncBN the double
// sums are what crosses ranks.
#include <algorithm>

#include "common.h"

namespace vae2 {

// ---------------------------------------------------- partial reductions ----
// Pixels per block for per-channel reductions: whole passes of the quad-path block
// (quad_rows(C) pixel rows x kApplyU pixels per thread), as many passes as keep the layer
// at <= 1024 blocks.  (Round 5 took ceil(P / 1024), at least 32, for every C: the narrow
// layers' blocks then ran one partial pass -- a 36-channel block covered 64 of the 112
// pixels its threads load, a 72-channel one 32 of 56 -- and the 18 / 36 / 72 backward
// reduce launches streamed at 0.34 of the HBM peak.)
static inline int quad_rows(int64_t C);
constexpr int kPassU = 4;  // = kApplyU (defined with the apply kernels below)
int g_bn_blocks = 1024;  // vae2_conv2d_set_tune key 19: blocks per layer (at most, whole passes)
// vae2_conv2d_set_tune key 20: the multi-layer apply kernels' resident-block budget R (0 =
// one workgroup per pixel chunk): a launch of T chunks runs ceil(T / ceil(T / R)) workgroups
// striding over them, so every workgroup does the same number of chunks in one round instead
// of a partial last round of blocks (the 18 / 36 / 72-channel launch: 2,165 chunks)
int g_bn_apply_res = 0;

static int64_t pix_per_block(int64_t P, int64_t C) {
  const int64_t pass = (int64_t)quad_rows(C) * kPassU;
  const int64_t n = ceil_div(P, (int64_t)g_bn_blocks * pass);
  return pass * (n > 0 ? n : 1);
}

// Mode 0: (sum x, sum x^2).  Mode 1: BN backward (sum g, sum g*xhat).
template <int MODE>
__global__ __launch_bounds__(256) void chan_partials_kernel(
    const float* __restrict__ x, Act xd, const float* __restrict__ dy, Act dyd,
    const float* __restrict__ y, Act yd, const float* __restrict__ save, int relu,
    int64_t ppb, float* __restrict__ part) {
  __shared__ float red[2][256];
  const int C = (int)xd.c;
  const int64_t P = xd.n * xd.h * xd.w;
  const int64_t p0 = blockIdx.x * ppb;
  int64_t p1 = p0 + ppb;
  if (p1 > P) p1 = P;
  const int rows = gridDim.x;
  const int tid = threadIdx.x;
  if (C <= 256) {
    const int R = 256 / C;  // pixels per step
    const int S = R * C;
    float s0 = 0.f, s1 = 0.f;
    if (tid < S) {
      const int c = tid % C;
      const int rr = tid / C;
      float mean = 0.f, invstd = 0.f, sc = 0.f, sh = 0.f;
      if (MODE == 1) { mean = save[c]; invstd = save[C + c]; sc = save[2 * C + c]; sh = save[3 * C + c]; }
      for (int64_t p = p0 + rr; p < p1; p += R) {
        float v = x[p * xd.ps + c];
        if (MODE == 0) {
          s0 += v;
          s1 += v * v;
        } else {
          float gv = dy[p * dyd.ps + c];
          if (relu && !((y ? y[p * yd.ps + c] : __builtin_fmaf(v, sc, sh)) > 0.f)) gv = 0.f;
          s0 += gv;
          s1 += gv * (v - mean) * invstd;
        }
      }
    }
    red[0][tid] = s0;
    red[1][tid] = s1;
    __syncthreads();
    if (tid < C) {
      float a = 0.f, b = 0.f;
      for (int i = 0; i < R; ++i) {
        a += red[0][tid + i * C];
        b += red[1][tid + i * C];
      }
      part[(int64_t)blockIdx.x * C + tid] = a;
      part[((int64_t)rows + blockIdx.x) * C + tid] = b;
    }
  } else {
    for (int c = tid; c < C; c += 256) {
      float s0 = 0.f, s1 = 0.f;
      float mean = 0.f, invstd = 0.f, sc = 0.f, sh = 0.f;
      if (MODE == 1) { mean = save[c]; invstd = save[C + c]; sc = save[2 * C + c]; sh = save[3 * C + c]; }
      for (int64_t p = p0; p < p1; ++p) {
        float v = x[p * xd.ps + c];
        if (MODE == 0) {
          s0 += v;
          s1 += v * v;
        } else {
          float gv = dy[p * dyd.ps + c];
          if (relu && !((y ? y[p * yd.ps + c] : __builtin_fmaf(v, sc, sh)) > 0.f)) gv = 0.f;
          s0 += gv;
          s1 += gv * (v - mean) * invstd;
        }
      }
      part[(int64_t)blockIdx.x * C + c] = s0;
      part[((int64_t)rows + blockIdx.x) * C + c] = s1;
    }
  }
}

// ------------------------------------------- channel-quad-stationary path ----
// Thread (r, q) of a block owns channels 4q..4q+3 and walks pixels r, r+rows, ...
// so per-channel coefficients stay in registers and every access is a 16-byte
// load/store of a contiguous pixel run.  Needs pixel strides % 4 == 0, 16-byte
// aligned bases and ceil(C/4) <= 256.  Channels >= C of the last quad are read
// (pixel padding, discarded) but never written.

__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }

// Per-channel coefficients of a channel quad: unconditional loads of clamped channels (a
// guarded load is branched around and waited for on its own), zero past C.
__device__ __forceinline__ f4 chan4(const float* a, int c, int C) {
  f4 v;
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = a[c + k < C ? c + k : C - 1];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = c + k < C ? v[k] : 0.f;
  return v;
}

__device__ __forceinline__ void st4(float* p, f4 v, int c, int C) {
  if (c + 4 <= C) {
    *reinterpret_cast<f4*>(p) = v;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c + k < C) p[k] = v[k];
  }
}

static inline int quad_rows(int64_t C) {
  const int c4 = (int)((C + 3) / 4);
  return c4 <= 256 ? 256 / c4 : 1;
}
constexpr int kApplyU = kPassU;  // pixels per thread in the apply kernels (2: 852 vs 861, 8: 841 vs 853 frames/s, round-4 A/B)

__global__ __launch_bounds__(256) void bn_apply_q_kernel(
    const float* __restrict__ x, Act xd, const float* __restrict__ save,
    const float* __restrict__ res, Act rd, float* __restrict__ y, Act yd, int relu,
    int rows) {
  const int C = (int)xd.c, c4 = (C + 3) >> 2;
  const int tid = threadIdx.x;
  if (tid >= rows * c4) return;
  const int r = tid / c4, c = 4 * (tid - r * c4);
  const f4 sc = chan4(save + 2 * C, c, C), sh = chan4(save + 3 * C, c, C);
  const int64_t P = xd.n * xd.h * xd.w;
  const int64_t pb = (int64_t)blockIdx.x * rows * kApplyU + r;
  f4 v[kApplyU], rv[kApplyU];
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    const int64_t p = pb + u * rows;
    if (p < P) {
      v[u] = ld4(x + p * xd.ps + c);
      if (res) rv[u] = ld4(res + p * rd.ps + c);
    }
  }
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    const int64_t p = pb + u * rows;
    if (p >= P) break;
    f4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float t = __builtin_fmaf(v[u][k], sc[k], sh[k]);
      if (res) t += rv[u][k];
      o[k] = (relu && t < 0.f) ? 0.f : t;  // NaN propagates (torch.relu)
    }
    st4(y + p * yd.ps + c, o, c, C);
  }
}

// Per-block partial rows: MODE 0 (sum x, sum x^2); MODE 1 (sum g, sum g*xhat) with
// g = dy masked by the ReLU of the forward output (y, or recomputed from x).
template <int MODE>
__global__ __launch_bounds__(256) void chan_partials_q_kernel(
    const float* __restrict__ x, Act xd, const float* __restrict__ dy, Act dyd,
    const float* __restrict__ y, Act yd, const float* __restrict__ save, int relu,
    int64_t ppb, int rows, float* __restrict__ part) {
  __shared__ float red[2][256 * 4];
  const int C = (int)xd.c, c4 = (C + 3) >> 2;
  const int tid = threadIdx.x;
  const int64_t P = xd.n * xd.h * xd.w;
  const int64_t p0 = blockIdx.x * ppb;
  int64_t p1 = p0 + ppb;
  if (p1 > P) p1 = P;
  f4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
  const int r = tid / c4, c = 4 * (tid - r * c4);
  if (tid < rows * c4) {
    f4 mean = {0.f, 0.f, 0.f, 0.f}, invstd = mean, sc = mean, sh = mean;
    if (MODE == 1) {
      mean = chan4(save, c, C);
      invstd = chan4(save + C, c, C);
      sc = chan4(save + 2 * C, c, C);
      sh = chan4(save + 3 * C, c, C);
    }
    int64_t p = p0 + r;
    for (; p + rows < p1; p += 2 * rows) {  // two pixels in flight
      const f4 xa = ld4(x + p * xd.ps + c), xb = ld4(x + (p + rows) * xd.ps + c);
      if (MODE == 0) {
        s0 += xa + xb;
        s1 += xa * xa + xb * xb;
      } else {
        f4 ga = ld4(dy + p * dyd.ps + c), gb = ld4(dy + (p + rows) * dyd.ps + c);
        f4 ya, yb;
        if (relu && y) {
          ya = ld4(y + p * yd.ps + c);
          yb = ld4(y + (p + rows) * yd.ps + c);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (relu) {
            const float ma = y ? ya[k] : __builtin_fmaf(xa[k], sc[k], sh[k]);
            const float mb = y ? yb[k] : __builtin_fmaf(xb[k], sc[k], sh[k]);
            if (!(ma > 0.f)) ga[k] = 0.f;
            if (!(mb > 0.f)) gb[k] = 0.f;
          }
          s0[k] += ga[k] + gb[k];
          s1[k] += ga[k] * (xa[k] - mean[k]) * invstd[k] + gb[k] * (xb[k] - mean[k]) * invstd[k];
        }
      }
    }
    if (p < p1) {
      const f4 xa = ld4(x + p * xd.ps + c);
      if (MODE == 0) {
        s0 += xa;
        s1 += xa * xa;
      } else {
        f4 ga = ld4(dy + p * dyd.ps + c);
        f4 ya;
        if (relu && y) ya = ld4(y + p * yd.ps + c);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (relu && !((y ? ya[k] : __builtin_fmaf(xa[k], sc[k], sh[k])) > 0.f)) ga[k] = 0.f;
          s0[k] += ga[k];
          s1[k] += ga[k] * (xa[k] - mean[k]) * invstd[k];
        }
      }
    }
  }
  // rows x (4*c4) layout: red[q][r * 4*c4 + c + k]
  if (tid < rows * c4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      red[0][r * 4 * c4 + c + k] = s0[k];
      red[1][r * 4 * c4 + c + k] = s1[k];
    }
  }
  __syncthreads();
  const int rowsC = (int)gridDim.x;
  for (int ch = tid; ch < C; ch += 256) {
    float a = 0.f, b = 0.f;
    for (int i = 0; i < rows; ++i) {
      a += red[0][i * 4 * c4 + ch];
      b += red[1][i * 4 * c4 + ch];
    }
    part[(int64_t)blockIdx.x * C + ch] = a;
    part[((int64_t)rowsC + blockIdx.x) * C + ch] = b;
  }
}

__global__ __launch_bounds__(256) void bn_bwd_apply_q_kernel(
    const float* __restrict__ dy, Act dyd, const float* __restrict__ y, Act yd,
    const float* __restrict__ x, Act xd, const float* __restrict__ save,
    const float* __restrict__ gamma, const double* __restrict__ sums, double count,
    int relu, float* __restrict__ dx, Act dxd, float* __restrict__ dres, Act rd, int rows) {
  const int C = (int)xd.c, c4 = (C + 3) >> 2;
  const int tid = threadIdx.x;
  if (tid >= rows * c4) return;
  const int r = tid / c4, c = 4 * (tid - r * c4);
  const float inv_n = (float)(1.0 / count);
  f4 mean, invstd, sc, sh, mg, mgx, k4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ch = c + k < C ? c + k : C - 1;
    mean[k] = save[ch];
    invstd[k] = save[C + ch];
    sc[k] = save[2 * C + ch];
    sh[k] = save[3 * C + ch];
    mg[k] = (float)sums[ch] * inv_n;
    mgx[k] = (float)sums[C + ch] * inv_n;
    k4[k] = (gamma ? gamma[ch] : 1.f) * invstd[k];
  }
  const int64_t P = xd.n * xd.h * xd.w;
  const int64_t pb = (int64_t)blockIdx.x * rows * kApplyU + r;
  f4 gv[kApplyU], xv[kApplyU], yv[kApplyU];
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    const int64_t p = pb + u * rows;
    if (p < P) {
      gv[u] = ld4(dy + p * dyd.ps + c);
      xv[u] = ld4(x + p * xd.ps + c);
      if (relu && y) yv[u] = ld4(y + p * yd.ps + c);
    }
  }
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    const int64_t p = pb + u * rows;
    if (p >= P) break;
    f4 g = gv[u], o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (relu && !((y ? yv[u][k] : __builtin_fmaf(xv[u][k], sc[k], sh[k])) > 0.f)) g[k] = 0.f;
      const float xh = (xv[u][k] - mean[k]) * invstd[k];
      o[k] = k4[k] * (g[k] - mg[k] - xh * mgx[k]);
    }
    if (dres) st4(dres + p * rd.ps + c, g, c, C);
    st4(dx + p * dxd.ps + c, o, c, C);
  }
}

// Thread tid's share of a per-channel reduction over partial rows (rows tid, tid+256,
// ... of column c; with `two`, also of the second block of rows): 4 rows' loads issued
// before their adds (latency, not bandwidth, bounds these small reductions), the adds
// in the same order as a plain strided loop, so the result is bit for bit the same.
// Range-checked buffer loads (rows past the end load 0): with `r < rows ? part[..] : 0`
// hipcc branched around each load and waited for it (16 dependent round trips per pass).
__device__ __forceinline__ void rows_sum2(const float* __restrict__ part, int64_t rows,
                                          int64_t C, int c, int tid, double& a, double& b,
                                          bool two = true) {
  constexpr int U = 8;
  const int64_t nb = (two ? 2 : 1) * rows * C * 4;
  const __amdgpu_buffer_rsrc_t pr = make_rsrc(part, (uint32_t)(nb < (int64_t)kOOB ? nb : kOOB));
  for (int64_t r0 = tid; r0 < rows; r0 += 256 * U) {
    float x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = r0 + 256 * u;
      x[u] = load1(pr, r < rows ? (uint32_t)((r * C + c) * 4) : kOOB);
      y[u] = load1(pr, two && r < rows ? (uint32_t)(((rows + r) * C + c) * 4) : kOOB);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (r0 + 256 * u < rows) {
        a += (double)x[u];
        b += (double)y[u];
      }
    }
  }
}

// One block per channel: sums[q][c] (+)= sum_rows part[q][row][c] in double.
__global__ __launch_bounds__(256) void partials_reduce_kernel(
    const float* __restrict__ part, int64_t rows, int64_t C, double* sums,
    int accumulate) {
  __shared__ double red[2][4];
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  double a = 0.0, b = 0.0;
  rows_sum2(part, rows, C, c, tid, a, b);
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = a;
    red[1][tid >> 6] = b;
  }
  __syncthreads();
  if (tid == 0) {
    double s0 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    double s1 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    if (accumulate) {
      sums[c] += s0;
      sums[C + c] += s1;
    } else {
      sums[c] = s0;
      sums[C + c] = s1;
    }
  }
}

// One block per channel: reduce partial rows (double, fixed order), then either
// finalize (MODE 0: mean/invstd/scale/shift + running stats) or write the sums and
// accumulate dgamma/dbeta (MODE 1: backward).  Used when no cross-rank exchange
// sits between the reduction and its consumer.
template <int MODE>
// mshift (optional): the partials are sums of (x - mshift[c]) (shifted statistics: no
// cancellation in E[x^2] - E[x]^2 when |mean| >> std); the mean gets the shift back.
__global__ __launch_bounds__(256) void reduce_then_kernel(
    const float* __restrict__ part, int64_t rows, int64_t C, double* sums, double count,
    const float* gamma, const float* beta, float* rmean, float* rvar, int64_t* nbt,
    float momentum, float eps, float* save, float* dgamma, float* dbeta,
    const float* mshift = nullptr) {
  __shared__ double red[2][4];
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  double a = 0.0, b = 0.0;
  rows_sum2(part, rows, C, c, tid, a, b);
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = a;
    red[1][tid >> 6] = b;
  }
  __syncthreads();
  if (tid != 0) return;
  const double s0 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  const double s1 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  sums[c] = s0;
  sums[C + c] = s1;
  if (MODE == 1) {
    if (dgamma) dgamma[c] += (float)s1;
    if (dbeta) dbeta[c] += (float)s0;
    return;
  }
  if (c == 0 && nbt) nbt[0] += 1;
  const double m0 = s0 / count;
  double var = s1 / count - m0 * m0;
  if (var < 0.0) var = 0.0;
  const double mean = m0 + (mshift ? (double)mshift[c] : 0.0);
  const double invstd = 1.0 / sqrt(var + (double)eps);
  const float gm = gamma ? gamma[c] : 1.f;
  const float bt = beta ? beta[c] : 0.f;
  save[c] = (float)mean;
  save[C + c] = (float)invstd;
  save[2 * C + c] = (float)(gm * invstd);
  save[3 * C + c] = (float)(bt - mean * (gm * invstd));
  if (rmean) {
    const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
    rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unbiased);
  }
}

__global__ void bn_finalize_kernel(const double* sums, double count,
                                   const float* gamma, const float* beta,
                                   float* rmean, float* rvar, int64_t* nbt,
                                   float momentum, float eps, int64_t C,
                                   float* save, const float* mshift = nullptr) {
  int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (c == 0 && nbt) nbt[0] += 1;
  if (c >= C) return;
  const double m0 = sums[c] / count;
  double var = sums[C + c] / count - m0 * m0;
  if (var < 0.0) var = 0.0;
  const double mean = m0 + (mshift ? (double)mshift[c] : 0.0);
  double invstd = 1.0 / sqrt(var + (double)eps);
  float g = gamma ? gamma[c] : 1.f;
  float b = beta ? beta[c] : 0.f;
  float scale = (float)(g * invstd);
  float shift = (float)(b - mean * (g * invstd));
  save[c] = (float)mean;
  save[C + c] = (float)invstd;
  save[2 * C + c] = scale;
  save[3 * C + c] = shift;
  if (rmean) {
    double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
    rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unbiased);
  }
}

__global__ void bn_eval_kernel(const float* gamma, const float* beta,
                               const float* rmean, const float* rvar, float eps,
                               int64_t C, float* save) {
  int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (c >= C) return;
  float invstd = 1.f / sqrtf(rvar[c] + eps);
  float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  save[c] = rmean[c];
  save[C + c] = invstd;
  save[2 * C + c] = g * invstd;
  save[3 * C + c] = b - rmean[c] * g * invstd;
}

// ------------------------------------------------------------- apply ----
__global__ __launch_bounds__(256) void bn_apply_kernel(
    const float* __restrict__ x, Act xd, const float* __restrict__ save,
    const float* __restrict__ res, Act rd, float* __restrict__ y, Act yd,
    int relu, FastDiv cdiv) {
  const uint32_t C = (uint32_t)xd.c;
  const uint32_t total = (uint32_t)(xd.n * xd.h * xd.w) * C;
  const float* scale = save + 2 * C;
  const float* shift = save + 3 * C;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t p = cdiv.div(i);
    uint32_t c = i - p * C;
    float v = __builtin_fmaf(x[(int64_t)p * xd.ps + c], scale[c], shift[c]);
    if (res) v += res[(int64_t)p * rd.ps + c];
    if (relu) v = v < 0.f ? 0.f : v;
    y[(int64_t)p * yd.ps + c] = v;
  }
}

// Vector path: C % 4 == 0, all pixel strides % 4 == 0, 16-byte aligned bases.
__global__ __launch_bounds__(256) void bn_apply_kernel_v4(
    const float* __restrict__ x, Act xd, const float* __restrict__ save,
    const float* __restrict__ res, Act rd, float* __restrict__ y, Act yd,
    int relu, FastDiv cdiv) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const uint32_t C4 = (uint32_t)xd.c / 4;
  const uint32_t C = (uint32_t)xd.c;
  const uint32_t total = (uint32_t)(xd.n * xd.h * xd.w) * C4;
  const float* scale = save + 2 * C;
  const float* shift = save + 3 * C;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t p = cdiv.div(i);
    uint32_t c = (i - p * C4) * 4;
    f4 v = *reinterpret_cast<const f4*>(x + (int64_t)p * xd.ps + c);
    f4 sc = *reinterpret_cast<const f4*>(scale + c);
    f4 sh = *reinterpret_cast<const f4*>(shift + c);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = __builtin_fmaf(v[k], sc[k], sh[k]);
    if (res) v += *reinterpret_cast<const f4*>(res + (int64_t)p * rd.ps + c);
    if (relu) {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = v[k] < 0.f ? 0.f : v[k];
    }
    *reinterpret_cast<f4*>(y + (int64_t)p * yd.ps + c) = v;
  }
}

__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const float* __restrict__ dy, Act dyd, const float* __restrict__ y, Act yd,
    const float* __restrict__ x, Act xd, const float* __restrict__ save,
    const float* __restrict__ gamma, const double* __restrict__ sums,
    double count, int relu, float* __restrict__ dx, Act dxd,
    float* __restrict__ dres, Act rd, FastDiv cdiv) {
  const uint32_t C = (uint32_t)xd.c;
  const uint32_t total = (uint32_t)(xd.n * xd.h * xd.w) * C;
  const float inv_n = (float)(1.0 / count);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t p = cdiv.div(i);
    uint32_t c = i - p * C;
    float g = dy[(int64_t)p * dyd.ps + c];
    const float xv = x[(int64_t)p * xd.ps + c];
    if (relu && !((y ? y[(int64_t)p * yd.ps + c]
                     : __builtin_fmaf(xv, save[2 * C + c], save[3 * C + c])) > 0.f))
      g = 0.f;
    if (dres) dres[(int64_t)p * rd.ps + c] = g;
    float mean = save[c], invstd = save[C + c];
    float mg = (float)sums[c] * inv_n;
    float mgx = (float)sums[C + c] * inv_n;
    float gm = gamma ? gamma[c] : 1.f;
    float xh = (xv - mean) * invstd;
    dx[(int64_t)p * dxd.ps + c] = gm * invstd * (g - mg - xh * mgx);
  }
}

__global__ void bn_param_grad_kernel(const double* sums, int64_t C,
                                     float* dgamma, float* dbeta) {
  int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (dgamma) dgamma[c] += (float)sums[C + c];
  if (dbeta) dbeta[c] += (float)sums[c];
}

__global__ __launch_bounds__(256) void colsum_to_float_kernel(
    const float* __restrict__ part, int64_t rows, int64_t C, float* out,
    int accumulate) {
  __shared__ double red[4];
  const int c = blockIdx.x, tid = threadIdx.x;
  double a = 0.0;
  {
    double b = 0.0;
    rows_sum2(part, rows, C, c, tid, a, b, false);
  }
  a = wave_sum_d(a);
  if ((tid & 63) == 0) red[tid >> 6] = a;
  __syncthreads();
  if (tid == 0) {
    float s = (float)(red[0] + red[1] + red[2] + red[3]);
    out[c] = accumulate ? out[c] + s : s;
  }
}

// ------------------------------------------------ multi-layer launches ----
// The independent BatchNorm layers of one HRNet depth level (the branches of a
// HighResolutionModule run in lockstep, the fuse convs of a module, the units of the
// transitions) share each launch: blocks are partitioned between the layers by
// prefix (blk0), each block runs the single-layer body on its own layer.  Up to
// kBnMaxLayers layers per launch (host splits larger groups).  Quad path only.
constexpr int kBnMaxLayers = 6;

struct BnLayer {
  const float* x;       // pre-BN activation r (the conv output)
  const float* a;       // forward: residual (or null); backward: y for the ReLU mask (or null)
  float* o;             // forward: y; backward: dx
  const float* dy;      // backward
  float* dres;          // backward: residual gradient (or null)
  float* part;          // backward reduce: partial rows [2][nblk][C]
  const float* save;    // mean, invstd, scale, shift
  const float* gamma;
  const double* sums;   // backward apply: global (sum g, sum g*xhat)
  const double* countp; // device count (SyncBN: all-reduced) or null -> count
  double count;
  int64_t P, ppb;
  int C, x_ps, a_ps, o_ps, dy_ps, dres_ps, relu, rows, blk0;
  int dres_acc;         // backward apply: dres += g instead of dres = g
  // residual through its own BatchNorm (no ReLU) whose output is never stored (the
  // Bottleneck's downsample shortcut): forward adds fma(rx, rscale, rshift); backward
  // writes that BN's partials (rpart) / input gradient (rdx) beside this layer's
  const float* rx;
  const float* rsave;
  const float* rgamma;
  float* rpart;
  const double* rsums;
  float* rdx;
  int rx_ps, rdx_ps;
  // ReLU mask, one byte per (pixel, channel quad) (bit k: channel 4q+k > 0): written by the
  // forward apply, read by the backward passes instead of y (1/16 of y's bytes)
  uint8_t* mk;
};

struct BnMulti {
  BnLayer L[kBnMaxLayers];
  int n;
  int v2;  // buffer-resource bodies (every extent < 2 GB; vae2_conv2d_set_tune key 8)
  int total;  // pixel chunks of the launch (apply kernels: workgroups stride over them)
};

// vae2_conv2d_set_tune key 8: 0 = the round-4 pointer-arithmetic BatchNorm bodies (A/B)
int g_bn_v2 = 1;

__device__ __forceinline__ int bn_layer_of(const BnMulti& m, int b) {
  int i = 0;
  while (i + 1 < m.n && b >= m.L[i + 1].blk0) ++i;
  return i;
}

__device__ __forceinline__ void bn_apply_body(const BnLayer& L, int blk) {
  const int C = L.C, c4 = (C + 3) >> 2;
  const int tid = threadIdx.x;
  if (tid >= L.rows * c4) return;
  const int r = tid / c4, c = 4 * (tid - r * c4);
  const f4 sc = chan4(L.save + 2 * C, c, C), sh = chan4(L.save + 3 * C, c, C);
  f4 rsc = {0.f, 0.f, 0.f, 0.f}, rsh = rsc;
  if (L.rx) { rsc = chan4(L.rsave + 2 * C, c, C); rsh = chan4(L.rsave + 3 * C, c, C); }
  const int64_t pb = (int64_t)blk * L.rows * kApplyU + r;
  // every load unconditional (pixels past P re-read pixel P-1, never stored) and the
  // uniform branches outside the pixel loop, so the loads of all pixels go out together
  f4 v[kApplyU], rv[kApplyU];
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    const int64_t p = pb + u * L.rows < L.P ? pb + u * L.rows : L.P - 1;
    v[u] = ld4(L.x + p * L.x_ps + c);
  }
  if (L.a) {
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) {
      const int64_t p = pb + u * L.rows < L.P ? pb + u * L.rows : L.P - 1;
      rv[u] = ld4(L.a + p * L.a_ps + c);
    }
  } else if (L.rx) {
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) {
      const int64_t p = pb + u * L.rows < L.P ? pb + u * L.rows : L.P - 1;
      rv[u] = ld4(L.rx + p * L.rx_ps + c);
    }
  }
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    const int64_t p = pb + u * L.rows;
    if (p >= L.P) break;
    f4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float t = __builtin_fmaf(v[u][k], sc[k], sh[k]);
      if (L.a) t += rv[u][k];
      // the residual BN's output, rounded as if stored, then added
      else if (L.rx) t += __builtin_fmaf(rv[u][k], rsc[k], rsh[k]);
      o[k] = (L.relu && t < 0.f) ? 0.f : t;  // NaN propagates (torch.relu)
    }
    st4(L.o + p * L.o_ps + c, o, c, C);
    if (L.mk)  // threshold_backward's test (y > 0: NaN and 0 cut the gradient)
      L.mk[p * c4 + (c >> 2)] = (uint8_t)((o[0] > 0.f) | ((o[1] > 0.f) << 1) |
                                          ((o[2] > 0.f) << 2) | ((o[3] > 0.f) << 3));
  }
}

// Buffer-resource form of bn_apply_body (same arithmetic; see bn_bwd_apply_body2).
__device__ __forceinline__ void bn_apply_body2(const BnLayer& L, int blk) {
  const int C = L.C, c4 = (C + 3) >> 2;
  const int tid = threadIdx.x;
  if (tid >= L.rows * c4) return;
  const int r = tid / c4, c = 4 * (tid - r * c4);
  const int nv = C - c < 4 ? C - c : 4;
  const bool part = (C & 3) != 0;
  const uint32_t P = (uint32_t)L.P;
  const uint32_t cb = (uint32_t)C * 4u;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(L.save, 4u * cb);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(L.x, P * (uint32_t)L.x_ps * 4u);
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(L.o, P * (uint32_t)L.o_ps * 4u);
  const uint32_t pb = (uint32_t)blk * (uint32_t)(L.rows * kApplyU) + (uint32_t)r;
  uint32_t pp[kApplyU];
  bool in[kApplyU];
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    const uint32_t p = pb + (uint32_t)(u * L.rows);
    in[u] = p < P;
    pp[u] = in[u] ? p : P - 1;
  }
  f4 v[kApplyU], rv[kApplyU];
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) v[u] = load4(rx, (pp[u] * (uint32_t)L.x_ps + (uint32_t)c) * 4u);
  if (L.a) {
    const __amdgpu_buffer_rsrc_t ra = make_rsrc(L.a, P * (uint32_t)L.a_ps * 4u);
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) rv[u] = load4(ra, (pp[u] * (uint32_t)L.a_ps + (uint32_t)c) * 4u);
  } else if (L.rx) {
    const __amdgpu_buffer_rsrc_t rr = make_rsrc(L.rx, P * (uint32_t)L.rx_ps * 4u);
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) rv[u] = load4(rr, (pp[u] * (uint32_t)L.rx_ps + (uint32_t)c) * 4u);
  }
  auto last_row4 = [&](__amdgpu_buffer_rsrc_t rr, uint32_t row) {
    f4 t;
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = load1(rr, row + 4u * (uint32_t)(c + k < C ? c + k : C - 1));
    return t;
  };
  const f4 sc = load4(rs, 2u * cb + 4u * (uint32_t)c), sh = last_row4(rs, 3u * cb);
  f4 rsc = {0.f, 0.f, 0.f, 0.f}, rsh = rsc;
  if (L.rx) {
    const __amdgpu_buffer_rsrc_t rrs = make_rsrc(L.rsave, 4u * cb);
    rsc = load4(rrs, 2u * cb + 4u * (uint32_t)c);
    rsh = last_row4(rrs, 3u * cb);
  }
  const __amdgpu_buffer_rsrc_t rm = make_rsrc(L.mk, L.mk ? P * (uint32_t)c4 : 0u);
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    f4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float t = __builtin_fmaf(v[u][k], sc[k], sh[k]);
      if (L.a) t += rv[u][k];
      else if (L.rx) t += __builtin_fmaf(rv[u][k], rsc[k], rsh[k]);
      o[k] = (L.relu && t < 0.f) ? 0.f : t;  // NaN propagates (torch.relu)
    }
    const uint32_t off = in[u] ? (pp[u] * (uint32_t)L.o_ps + (uint32_t)c) * 4u : kOOB;
    if (part) store_quad(ro, off, o, nv);
    else store4(ro, off, o);
    if (L.mk)  // threshold_backward's test (y > 0: NaN and 0 cut the gradient)
      __builtin_amdgcn_raw_buffer_store_b8(
          (uint8_t)((o[0] > 0.f) | ((o[1] > 0.f) << 1) | ((o[2] > 0.f) << 2) | ((o[3] > 0.f) << 3)),
          rm, in[u] ? pp[u] * (uint32_t)c4 + (uint32_t)(c >> 2) : kOOB, 0, 0);
  }
}

__global__ __launch_bounds__(256) void bn_apply_multi_kernel(BnMulti m) {
  for (int b = blockIdx.x; b < m.total; b += gridDim.x) {  // (once unless key 20 is set)
    const int i = bn_layer_of(m, b);
    bn_apply_body2(m.L[i], b - m.L[i].blk0);
  }
}

__global__ __launch_bounds__(256) void bn_apply_multi_r4_kernel(BnMulti m) {
  const int i = bn_layer_of(m, blockIdx.x);
  bn_apply_body(m.L[i], blockIdx.x - m.L[i].blk0);
}

// Backward partials (sum g, sum g*xhat) of one layer's pixel range blk*ppb ...
__device__ __forceinline__ void bn_bwd_reduce_body(const BnLayer& L, int blk, int nblk,
                                                   float* red0, float* red1) {
  const int C = L.C, c4 = (C + 3) >> 2;
  const int tid = threadIdx.x;
  const int64_t p0 = blk * L.ppb;
  int64_t p1 = p0 + L.ppb;
  if (p1 > L.P) p1 = L.P;
  f4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f}, s2 = s0;
  const int r = tid / c4, c = 4 * (tid - r * c4);
  const uint8_t* mk = L.relu ? L.mk : nullptr;  // stored mask, else y, else from x
  const float* y = L.relu && !mk ? L.a : nullptr;
  const bool rb = L.rx != nullptr;  // + the residual BN's sum g * xhat_r (same g)
  if (tid < L.rows * c4) {
    const f4 mean = chan4(L.save, c, C), invstd = chan4(L.save + C, c, C);
    const f4 sc = chan4(L.save + 2 * C, c, C), sh = chan4(L.save + 3 * C, c, C);
    f4 rmean = s0, rinv = s0;
    if (rb) { rmean = chan4(L.rsave, c, C); rinv = chan4(L.rsave + C, c, C); }
    // kApplyU pixels' loads in flight per thread, then their math in pixel order (the
    // same accumulation order as one pixel at a time)
    for (int64_t pb = p0 + r; pb < p1; pb += (int64_t)kApplyU * L.rows) {
      f4 xv[kApplyU], gv[kApplyU], yv[kApplyU], rv[kApplyU];
      uint32_t mv[kApplyU];
      // unconditional loads (pixels past p1 re-read p1 - 1, not summed), uniform branches
      // outside the pixel loop: all pixels' loads in flight together
      int64_t pp[kApplyU];
#pragma unroll
      for (int u = 0; u < kApplyU; ++u) pp[u] = pb + u * L.rows < p1 ? pb + u * L.rows : p1 - 1;
#pragma unroll
      for (int u = 0; u < kApplyU; ++u) {
        xv[u] = ld4(L.x + pp[u] * L.x_ps + c);
        gv[u] = ld4(L.dy + pp[u] * L.dy_ps + c);
      }
      if (y) {
#pragma unroll
        for (int u = 0; u < kApplyU; ++u) yv[u] = ld4(y + pp[u] * L.a_ps + c);
      }
      if (mk) {
#pragma unroll
        for (int u = 0; u < kApplyU; ++u) mv[u] = mk[pp[u] * c4 + (c >> 2)];
      }
      if (rb) {
#pragma unroll
        for (int u = 0; u < kApplyU; ++u) rv[u] = ld4(L.rx + pp[u] * L.rx_ps + c);
      }
#pragma unroll
      for (int u = 0; u < kApplyU; ++u) {
        if (pb + u * L.rows >= p1) break;
        const f4 xa = xv[u];
        f4 ga = gv[u];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (L.relu && !(mk ? ((mv[u] >> k) & 1u) != 0
                             : (y ? yv[u][k] : __builtin_fmaf(xa[k], sc[k], sh[k])) > 0.f))
            ga[k] = 0.f;
          s0[k] += ga[k];
          s1[k] += ga[k] * (xa[k] - mean[k]) * invstd[k];
          if (rb) s2[k] += ga[k] * (rv[u][k] - rmean[k]) * rinv[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      red0[r * 4 * c4 + c + k] = s0[k];
      red1[r * 4 * c4 + c + k] = s1[k];
    }
  }
  __syncthreads();
  for (int ch = tid; ch < C; ch += 256) {
    float a = 0.f, b = 0.f;
    for (int i = 0; i < L.rows; ++i) {
      a += red0[i * 4 * c4 + ch];
      b += red1[i * 4 * c4 + ch];
    }
    L.part[(int64_t)blk * C + ch] = a;
    L.part[((int64_t)nblk + blk) * C + ch] = b;
    if (rb) L.rpart[(int64_t)blk * C + ch] = a;  // the residual BN's sum g: the same sum
  }
  if (!rb) return;
  __syncthreads();
  if (tid < L.rows * c4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) red1[r * 4 * c4 + c + k] = s2[k];
  }
  __syncthreads();
  for (int ch = tid; ch < C; ch += 256) {
    float b = 0.f;
    for (int i = 0; i < L.rows; ++i) b += red1[i * 4 * c4 + ch];
    L.rpart[((int64_t)nblk + blk) * C + ch] = b;
  }
}

// Buffer-resource form of bn_bwd_reduce_body (same arithmetic and summation order),
// specialised like bn_bwd_apply_body2 (ACT: ReLU mask source, RB: residual BatchNorm).
template <int ACT, bool RB>
__device__ __forceinline__ void bn_bwd_reduce_body2(const BnLayer& L, int blk, int nblk,
                                                   float* red0, float* red1) {
  const int C = L.C, c4 = (C + 3) >> 2;
  const int tid = threadIdx.x;
  const int64_t p0 = blk * L.ppb;
  int64_t p1 = p0 + L.ppb;
  if (p1 > L.P) p1 = L.P;
  f4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f}, s2 = s0;
  const int r = tid / c4, c = 4 * (tid - r * c4);
  // stored mask, else y, else from x (ACT 0 / 1 / 2 fixed at compile time, 3 per layer)
  const uint8_t* mk = L.relu && (ACT == 1 || ACT == 3) ? L.mk : nullptr;
  const float* y = L.relu && (ACT == 2 || (ACT == 3 && !mk)) ? L.a : nullptr;
  const bool rb = RB && L.rx != nullptr;  // + the residual BN's sum g * xhat_r (same g)
  const uint32_t P = (uint32_t)L.P;
  const __amdgpu_buffer_rsrc_t rxx = make_rsrc(L.x, P * (uint32_t)L.x_ps * 4u);
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc(L.dy, P * (uint32_t)L.dy_ps * 4u);
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(y, y ? P * (uint32_t)L.a_ps * 4u : 0u);
  const __amdgpu_buffer_rsrc_t rm = make_rsrc(mk, mk ? P * (uint32_t)c4 : 0u);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(L.rx, rb ? P * (uint32_t)L.rx_ps * 4u : 0u);
  if (tid < L.rows * c4) {
    const f4 mean = chan4(L.save, c, C), invstd = chan4(L.save + C, c, C);
    const f4 sc = chan4(L.save + 2 * C, c, C), sh = chan4(L.save + 3 * C, c, C);
    f4 rmean = s0, rinv = s0;
    if (rb) { rmean = chan4(L.rsave, c, C); rinv = chan4(L.rsave + C, c, C); }
    // kApplyU pixels' loads in flight per thread, then their math in pixel order (the
    // same accumulation order as one pixel at a time)
    for (int64_t pb = p0 + r; pb < p1; pb += (int64_t)kApplyU * L.rows) {
      f4 xv[kApplyU], gv[kApplyU], yv[kApplyU], rv[kApplyU];
      uint32_t mv[kApplyU];
      // unconditional loads (pixels past p1 re-read p1 - 1, not summed), uniform branches
      // outside the pixel loop: all pixels' loads in flight together
      uint32_t pp[kApplyU];
#pragma unroll
      for (int u = 0; u < kApplyU; ++u)
        pp[u] = (uint32_t)(pb + u * L.rows < p1 ? pb + u * L.rows : p1 - 1);
#pragma unroll
      for (int u = 0; u < kApplyU; ++u) {
        xv[u] = load4(rxx, (pp[u] * (uint32_t)L.x_ps + (uint32_t)c) * 4u);
        gv[u] = load4(rdy, (pp[u] * (uint32_t)L.dy_ps + (uint32_t)c) * 4u);
      }
      if (y) {
#pragma unroll
        for (int u = 0; u < kApplyU; ++u) yv[u] = load4(ry, (pp[u] * (uint32_t)L.a_ps + (uint32_t)c) * 4u);
      }
      if (mk) {
#pragma unroll
        for (int u = 0; u < kApplyU; ++u) mv[u] = load_u8(rm, pp[u] * (uint32_t)c4 + (uint32_t)(c >> 2));
      }
      if (rb) {
#pragma unroll
        for (int u = 0; u < kApplyU; ++u) rv[u] = load4(rr, (pp[u] * (uint32_t)L.rx_ps + (uint32_t)c) * 4u);
      }
#pragma unroll
      for (int u = 0; u < kApplyU; ++u) {
        if (pb + u * L.rows >= p1) break;
        const f4 xa = xv[u];
        f4 ga = gv[u];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (L.relu && !(mk ? ((mv[u] >> k) & 1u) != 0
                             : (y ? yv[u][k] : __builtin_fmaf(xa[k], sc[k], sh[k])) > 0.f))
            ga[k] = 0.f;
          s0[k] += ga[k];
          s1[k] += ga[k] * (xa[k] - mean[k]) * invstd[k];
          if (rb) s2[k] += ga[k] * (rv[u][k] - rmean[k]) * rinv[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      red0[r * 4 * c4 + c + k] = s0[k];
      red1[r * 4 * c4 + c + k] = s1[k];
    }
  }
  __syncthreads();
  for (int ch = tid; ch < C; ch += 256) {
    float a = 0.f, b = 0.f;
    for (int i = 0; i < L.rows; ++i) {
      a += red0[i * 4 * c4 + ch];
      b += red1[i * 4 * c4 + ch];
    }
    L.part[(int64_t)blk * C + ch] = a;
    L.part[((int64_t)nblk + blk) * C + ch] = b;
    if (rb) L.rpart[(int64_t)blk * C + ch] = a;  // the residual BN's sum g: the same sum
  }
  if (!rb) return;
  __syncthreads();
  if (tid < L.rows * c4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) red1[r * 4 * c4 + c + k] = s2[k];
  }
  __syncthreads();
  for (int ch = tid; ch < C; ch += 256) {
    float b = 0.f;
    for (int i = 0; i < L.rows; ++i) b += red1[i * 4 * c4 + ch];
    L.rpart[((int64_t)nblk + blk) * C + ch] = b;
  }
}

// nblk of layer i = blk0[i+1] - blk0[i] (the last: gridDim.x - blk0)
template <int ACT, bool RB>
__global__ __launch_bounds__(256) void bn_bwd_reduce_multi_kernel(BnMulti m) {
  __shared__ float red[2][256 * 4];
  const int i = bn_layer_of(m, blockIdx.x);
  const int nblk = (i + 1 < m.n ? m.L[i + 1].blk0 : (int)gridDim.x) - m.L[i].blk0;
  bn_bwd_reduce_body2<ACT, RB>(m.L[i], blockIdx.x - m.L[i].blk0, nblk, red[0], red[1]);
}

static void bwd_reduce_launch(const BnMulti& m, unsigned blocks, hipStream_t st) {
  int act = -1;
  bool rb = false;
  for (int j = 0; j < m.n; ++j) {
    const BnLayer& L = m.L[j];
    const int a = !L.relu ? 0 : (L.mk ? 1 : (L.a ? 2 : 0));
    act = act < 0 ? a : (act == a ? act : 3);
    rb = rb || L.rx;
  }
#define BWR(A)                                                                                    \
  do {                                                                                            \
    if (rb) VAE2_LAUNCH((bn_bwd_reduce_multi_kernel<A, true>), dim3(blocks), dim3(256), 0, st, m); \
    else VAE2_LAUNCH((bn_bwd_reduce_multi_kernel<A, false>), dim3(blocks), dim3(256), 0, st, m);   \
  } while (0)
  switch (act) {
    case 0: BWR(0); break;
    case 1: BWR(1); break;
    case 2: BWR(2); break;
    default: BWR(3); break;
  }
#undef BWR
}

__global__ __launch_bounds__(256) void bn_bwd_reduce_multi_r4_kernel(BnMulti m) {
  __shared__ float red[2][256 * 4];
  const int i = bn_layer_of(m, blockIdx.x);
  const int nblk = (i + 1 < m.n ? m.L[i + 1].blk0 : (int)gridDim.x) - m.L[i].blk0;
  bn_bwd_reduce_body(m.L[i], blockIdx.x - m.L[i].blk0, nblk, red[0], red[1]);
}

__device__ __forceinline__ void bn_bwd_apply_body(const BnLayer& L, int blk) {
  const int C = L.C, c4 = (C + 3) >> 2;
  const int tid = threadIdx.x;
  if (tid >= L.rows * c4) return;
  const int r = tid / c4, c = 4 * (tid - r * c4);
  const uint8_t* mk = L.relu ? L.mk : nullptr;  // stored mask, else y, else from x
  const float* y = L.relu && !mk ? L.a : nullptr;
  const bool rb = L.rx != nullptr;
  // the pixels' loads first (unconditional: pixels past P re-read P-1, never stored; the
  // uniform branches outside the pixel loop), then the per-channel coefficients
  const int64_t pb = (int64_t)blk * L.rows * kApplyU + r;
  f4 gv[kApplyU], xv[kApplyU], yv[kApplyU], rxv[kApplyU];
  uint32_t mv[kApplyU];
  int64_t pp[kApplyU];
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) pp[u] = pb + u * L.rows < L.P ? pb + u * L.rows : L.P - 1;
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    gv[u] = ld4(L.dy + pp[u] * L.dy_ps + c);
    xv[u] = ld4(L.x + pp[u] * L.x_ps + c);
  }
  if (y) {
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) yv[u] = ld4(y + pp[u] * L.a_ps + c);
  }
  if (mk) {
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) mv[u] = mk[pp[u] * c4 + (c >> 2)];
  }
  if (rb) {
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) rxv[u] = ld4(L.rx + pp[u] * L.rx_ps + c);
  }
  f4 dv[kApplyU];  // the residual gradient accumulated onto (dres_acc)
  if (L.dres && L.dres_acc) {
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) dv[u] = ld4(L.dres + pp[u] * L.dres_ps + c);
  }
  const double count = L.countp ? *L.countp : L.count;
  const float inv_n = (float)(1.0 / count);
  f4 mean, invstd, sc, sh, mg, mgx, k4;
  f4 rmean = {0.f, 0.f, 0.f, 0.f}, rinv = rmean, rmg = rmean, rmgx = rmean, rk4 = rmean;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ch = c + k < C ? c + k : C - 1;
    mean[k] = L.save[ch];
    invstd[k] = L.save[C + ch];
    sc[k] = L.save[2 * C + ch];
    sh[k] = L.save[3 * C + ch];
    mg[k] = (float)L.sums[ch] * inv_n;
    mgx[k] = (float)L.sums[C + ch] * inv_n;
    k4[k] = (L.gamma ? L.gamma[ch] : 1.f) * invstd[k];
    if (rb) {
      rmean[k] = L.rsave[ch];
      rinv[k] = L.rsave[C + ch];
      rmg[k] = (float)L.rsums[ch] * inv_n;
      rmgx[k] = (float)L.rsums[C + ch] * inv_n;
      rk4[k] = (L.rgamma ? L.rgamma[ch] : 1.f) * rinv[k];
    }
  }
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    const int64_t p = pb + u * L.rows;
    if (p >= L.P) break;
    f4 g = gv[u], o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (L.relu && !(mk ? ((mv[u] >> k) & 1u) != 0
                         : (y ? yv[u][k] : __builtin_fmaf(xv[u][k], sc[k], sh[k])) > 0.f))
        g[k] = 0.f;
      const float xh = (xv[u][k] - mean[k]) * invstd[k];
      o[k] = k4[k] * (g[k] - mg[k] - xh * mgx[k]);
    }
    if (L.dres) {
      float* dr = L.dres + p * L.dres_ps + c;
      st4(dr, L.dres_acc ? g + dv[u] : g, c, C);
    }
    st4(L.o + p * L.o_ps + c, o, c, C);
    if (rb) {  // the residual BN's input gradient from the same g (bn_bwd_apply's formula)
      f4 ro;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float xh = (rxv[u][k] - rmean[k]) * rinv[k];
        ro[k] = rk4[k] * (g[k] - rmg[k] - xh * rmgx[k]);
      }
      st4(L.rdx + p * L.rdx_ps + c, ro, c, C);
    }
  }
}

// Buffer-resource form of bn_bwd_apply_body (same arithmetic, element for element): 32-bit
// byte offsets instead of 64-bit pointer math, 16-byte coefficient loads (out-of-range
// lanes read 0), pixels past P clamped for the loads and dropped for the stores
// (out-of-range offsets), partial channel quads stored by store_quad -- no per-lane
// branches.  SQ PMC of the round-4 form on the 18 / 36 / 72-channel launches: 405 VALU +
// 308 SALU instructions per wave (64-bit addresses, per-channel scalar coefficient loads,
// exec-mask branches around the partial-quad stores), 40 % of wave cycles in issue stalls.
// Every tensor extent < 2 GB (host check, bn_multi_launch).
// ACT (compile time, so the unused operand arrays cost no registers): how the ReLU mask is
// known -- 0 recomputed from x (or no ReLU), 1 mask bytes, 2 stored y, 3 decided per layer;
// RB: some layer has a residual BatchNorm (rx); DACC: some layer accumulates onto dres.
// (The all-features body held 158 VGPRs: 3 workgroups per CU, a narrow 3-layer launch of
// ~2,200 workgroups ran in ~3 rounds.)
template <int ACT, bool RB, bool DACC>
__device__ __forceinline__ void bn_bwd_apply_body2(const BnLayer& L, int blk) {
  const int C = L.C, c4 = (C + 3) >> 2;
  const int tid = threadIdx.x;
  if (tid >= L.rows * c4) return;
  const int r = tid / c4, c = 4 * (tid - r * c4);
  const int nv = C - c < 4 ? C - c : 4;  // valid channels of this quad
  const bool part = (C & 3) != 0;        // (uniform) some quad is partial
  const uint32_t P = (uint32_t)L.P;
  const bool relu = L.relu != 0;
  const bool usemk = relu && (ACT == 1 || (ACT == 3 && L.mk != nullptr));
  const bool usey = relu && (ACT == 2 || (ACT == 3 && L.mk == nullptr && L.a != nullptr));
  const bool rb = RB && L.rx != nullptr;
  const bool dres = L.dres != nullptr;
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc(L.dy, P * (uint32_t)L.dy_ps * 4u);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(L.x, P * (uint32_t)L.x_ps * 4u);
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(L.o, P * (uint32_t)L.o_ps * 4u);
  const uint32_t pb = (uint32_t)blk * (uint32_t)(L.rows * kApplyU) + (uint32_t)r;
  uint32_t pp[kApplyU];
  bool in[kApplyU];
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    const uint32_t p = pb + (uint32_t)(u * L.rows);
    in[u] = p < P;
    pp[u] = in[u] ? p : P - 1;
  }
  f4 gv[kApplyU], xv[kApplyU], yv[kApplyU], rxv[kApplyU], dv[kApplyU];
  uint32_t mv[kApplyU];
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    gv[u] = load4(rdy, (pp[u] * (uint32_t)L.dy_ps + (uint32_t)c) * 4u);
    xv[u] = load4(rx, (pp[u] * (uint32_t)L.x_ps + (uint32_t)c) * 4u);
  }
  if ((ACT == 2 || ACT == 3) && usey) {
    const __amdgpu_buffer_rsrc_t ry = make_rsrc(L.a, P * (uint32_t)L.a_ps * 4u);
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) yv[u] = load4(ry, (pp[u] * (uint32_t)L.a_ps + (uint32_t)c) * 4u);
  }
  if ((ACT == 1 || ACT == 3) && usemk) {
    const __amdgpu_buffer_rsrc_t rm = make_rsrc(L.mk, P * (uint32_t)c4);
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) mv[u] = load_u8(rm, pp[u] * (uint32_t)c4 + (uint32_t)(c >> 2));
  }
  if (rb) {
    const __amdgpu_buffer_rsrc_t rr = make_rsrc(L.rx, P * (uint32_t)L.rx_ps * 4u);
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) rxv[u] = load4(rr, (pp[u] * (uint32_t)L.rx_ps + (uint32_t)c) * 4u);
  }
  const __amdgpu_buffer_rsrc_t rdr = make_rsrc(L.dres, dres ? P * (uint32_t)L.dres_ps * 4u : 0u);
  const bool dacc = DACC && dres && L.dres_acc;
  if (dacc) {
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) dv[u] = load4(rdr, (pp[u] * (uint32_t)L.dres_ps + (uint32_t)c) * 4u);
  }
  // per-channel coefficients: 16-byte loads of the quad where they stay inside the buffer
  // (a partial quad then reads the next coefficient row: only its dropped lanes use those),
  // per-channel loads of clamped channels for the last row of a buffer (a 16-byte load that
  // crosses the end of the range returns 0 in every lane)
  const uint32_t cb = (uint32_t)C * 4u, qb = (uint32_t)c * 4u;
  auto last_row4 = [&](__amdgpu_buffer_rsrc_t rr, uint32_t row) {
    f4 v;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = load1(rr, row + 4u * (uint32_t)(c + k < C ? c + k : C - 1));
    return v;
  };
  auto last_row_d4 = [&](__amdgpu_buffer_rsrc_t rr, uint32_t row, float scale) {
    f4 v;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t o = row + 8u * (uint32_t)(c + k < C ? c + k : C - 1);
      const u32x2 b = __builtin_amdgcn_raw_buffer_load_b64(rr, o, 0, 0);
      v[k] = (float)__builtin_bit_cast(double, b) * scale;
    }
    return v;
  };
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(L.save, 4u * cb);
  const f4 mean = load4(rs, qb), invstd = load4(rs, cb + qb);
  const f4 sc = load4(rs, 2u * cb + qb), sh = last_row4(rs, 3u * cb);
  const __amdgpu_buffer_rsrc_t rsum = make_rsrc(L.sums, 2u * cb * 2u);
  const d2 s01 = load_d2(rsum, 2u * qb), s23 = load_d2(rsum, 2u * qb + 16u);
  f4 gam = {1.f, 1.f, 1.f, 1.f};
  if (L.gamma) gam = last_row4(make_rsrc(L.gamma, cb), 0u);
  const double count = L.countp ? *L.countp : L.count;
  const float inv_n = (float)(1.0 / count);
  const f4 mg = {(float)s01[0] * inv_n, (float)s01[1] * inv_n, (float)s23[0] * inv_n, (float)s23[1] * inv_n};
  const f4 mgx = last_row_d4(rsum, 2u * cb, inv_n);
  const f4 k4 = gam * invstd;
  f4 rmean = {0.f, 0.f, 0.f, 0.f}, rinv = rmean, rmg = rmean, rmgx = rmean, rk4 = rmean;
  if (rb) {
    const __amdgpu_buffer_rsrc_t rrs = make_rsrc(L.rsave, 4u * cb);
    rmean = load4(rrs, qb);
    rinv = load4(rrs, cb + qb);
    const __amdgpu_buffer_rsrc_t rrsum = make_rsrc(L.rsums, 2u * cb * 2u);
    const d2 a01 = load_d2(rrsum, 2u * qb), a23 = load_d2(rrsum, 2u * qb + 16u);
    rmg = f4{(float)a01[0] * inv_n, (float)a01[1] * inv_n, (float)a23[0] * inv_n, (float)a23[1] * inv_n};
    rmgx = last_row_d4(rrsum, 2u * cb, inv_n);
    f4 rgam = {1.f, 1.f, 1.f, 1.f};
    if (L.rgamma) rgam = last_row4(make_rsrc(L.rgamma, cb), 0u);
    rk4 = rgam * rinv;
  }
  const __amdgpu_buffer_rsrc_t rrdx = make_rsrc(L.rdx, rb ? P * (uint32_t)L.rdx_ps * 4u : 0u);
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    f4 g = gv[u], o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bool pos;
      if ((ACT == 1 || ACT == 3) && usemk) pos = ((mv[u] >> k) & 1u) != 0;
      else if ((ACT == 2 || ACT == 3) && usey) pos = yv[u][k] > 0.f;
      else pos = __builtin_fmaf(xv[u][k], sc[k], sh[k]) > 0.f;
      if (relu && !pos) g[k] = 0.f;
      const float xh = (xv[u][k] - mean[k]) * invstd[k];
      o[k] = k4[k] * (g[k] - mg[k] - xh * mgx[k]);
    }
    const uint32_t po = in[u] ? pp[u] : 0x7fffffffu;  // pixels past P: dropped stores
    auto off = [&](int ps) { return in[u] ? (po * (uint32_t)ps + (uint32_t)c) * 4u : kOOB; };
    if (dres) {
      const f4 dr = dacc ? g + dv[u] : g;
      if (part) store_quad(rdr, off(L.dres_ps), dr, nv);
      else store4(rdr, off(L.dres_ps), dr);
    }
    if (part) store_quad(ro, off(L.o_ps), o, nv);
    else store4(ro, off(L.o_ps), o);
    if (rb) {  // the residual BN's input gradient from the same g (bn_bwd_apply's formula)
      f4 rdv;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float xh = (rxv[u][k] - rmean[k]) * rinv[k];
        rdv[k] = rk4[k] * (g[k] - rmg[k] - xh * rmgx[k]);
      }
      if (part) store_quad(rrdx, off(L.rdx_ps), rdv, nv);
      else store4(rrdx, off(L.rdx_ps), rdv);
    }
  }
}

template <int ACT, bool RB, bool DACC>
__global__ __launch_bounds__(256) void bn_bwd_apply_multi_kernel(BnMulti m) {
  for (int b = blockIdx.x; b < m.total; b += gridDim.x) {  // (once unless key 20 is set)
    const int i = bn_layer_of(m, b);
    bn_bwd_apply_body2<ACT, RB, DACC>(m.L[i], b - m.L[i].blk0);
  }
}

// The specialisation of a launch: the union of its layers' features.
static void bwd_apply_launch(const BnMulti& m, unsigned blocks, hipStream_t st) {
  int act = -1;
  bool rb = false, dacc = false;
  for (int j = 0; j < m.n; ++j) {
    const BnLayer& L = m.L[j];
    const int a = !L.relu ? 0 : (L.mk ? 1 : (L.a ? 2 : 0));
    act = act < 0 ? a : (act == a ? act : 3);
    rb = rb || L.rx;
    dacc = dacc || (L.dres && L.dres_acc);
  }
#define BWA(A)                                                                                  \
  do {                                                                                          \
    if (rb && dacc) VAE2_LAUNCH((bn_bwd_apply_multi_kernel<A, true, true>), dim3(blocks), dim3(256), 0, st, m); \
    else if (rb) VAE2_LAUNCH((bn_bwd_apply_multi_kernel<A, true, false>), dim3(blocks), dim3(256), 0, st, m);   \
    else if (dacc) VAE2_LAUNCH((bn_bwd_apply_multi_kernel<A, false, true>), dim3(blocks), dim3(256), 0, st, m); \
    else VAE2_LAUNCH((bn_bwd_apply_multi_kernel<A, false, false>), dim3(blocks), dim3(256), 0, st, m);          \
  } while (0)
  switch (act) {
    case 0: BWA(0); break;
    case 1: BWA(1); break;
    case 2: BWA(2); break;
    default: BWA(3); break;
  }
#undef BWA
}

__global__ __launch_bounds__(256) void bn_bwd_apply_multi_r4_kernel(BnMulti m) {
  const int i = bn_layer_of(m, blockIdx.x);
  bn_bwd_apply_body(m.L[i], blockIdx.x - m.L[i].blk0);
}

// One block per (layer, channel): reduce the layer's partial rows in double (fixed
// order), then MODE 0: finalize (+ running statistics); MODE 1: sums + dgamma/dbeta
// (backward); MODE 2: sums only (SyncBN, exchanged before vae2_bn_multi_finalize).
struct FinLayer {
  const float* part;
  double* sums;
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  int64_t* nbt;
  float* save;
  float* dgamma;
  float* dbeta;
  const double* countp;
  double count;
  int64_t rows;
  float momentum, eps;
  int C, blk0;
};

struct FinMulti {
  FinLayer L[kBnMaxLayers];
  int n;
};

__device__ __forceinline__ void bn_finalize_channel(const FinLayer& L, int c, double s0,
                                                    double s1) {
  const double count = L.countp ? *L.countp : L.count;
  if (c == 0 && L.nbt) L.nbt[0] += 1;
  const double mean = s0 / count;
  double var = s1 / count - mean * mean;
  if (var < 0.0) var = 0.0;
  const double invstd = 1.0 / sqrt(var + (double)L.eps);
  const float gm = L.gamma ? L.gamma[c] : 1.f;
  const float bt = L.beta ? L.beta[c] : 0.f;
  L.save[c] = (float)mean;
  L.save[L.C + c] = (float)invstd;
  L.save[2 * L.C + c] = (float)(gm * invstd);
  L.save[3 * L.C + c] = (float)(bt - mean * (gm * invstd));
  if (L.rmean) {
    const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
    L.rmean[c] = (float)((1.0 - L.momentum) * L.rmean[c] + L.momentum * mean);
    L.rvar[c] = (float)((1.0 - L.momentum) * L.rvar[c] + L.momentum * unbiased);
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void reduce_then_multi_kernel(FinMulti m) {
  __shared__ double red[2][4];
  int i = 0;
  while (i + 1 < m.n && (int)blockIdx.x >= m.L[i + 1].blk0) ++i;
  const FinLayer& L = m.L[i];
  const int c = blockIdx.x - L.blk0;
  const int tid = threadIdx.x;
  double a = 0.0, b = 0.0;
  rows_sum2(L.part, L.rows, L.C, c, tid, a, b);
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = a;
    red[1][tid >> 6] = b;
  }
  __syncthreads();
  if (tid != 0) return;
  const double s0 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  const double s1 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  L.sums[c] = s0;
  L.sums[L.C + c] = s1;
  if (MODE == 1) {
    if (L.dgamma) L.dgamma[c] += (float)s1;
    if (L.dbeta) L.dbeta[c] += (float)s0;
  } else if (MODE == 0) {
    bn_finalize_channel(L, c, s0, s1);
  }
}

// From (all-reduced) sums: one block per layer, threads over channels.
__global__ __launch_bounds__(256) void bn_finalize_multi_kernel(FinMulti m) {
  const FinLayer& L = m.L[blockIdx.x];
  for (int c = threadIdx.x; c < L.C; c += 256) bn_finalize_channel(L, c, L.sums[c], L.sums[L.C + c]);
}

static bool v4_ok(const void* p, int64_t ps) {
  return ((uintptr_t)p % 16 == 0) && (ps % 4 == 0);
}

static bool quad_ok(int64_t c) { return (c + 3) / 4 <= 256; }

int bias_grad_from_partials(const float* partials, int64_t rows, int64_t c,
                            float* dbias, int accumulate, void* stream) {
  VAE2_LAUNCH(colsum_to_float_kernel, dim3((unsigned)c), dim3(256), 0,
                     as_stream(stream), partials, rows, c, dbias, accumulate);
  return check_launch("bias_grad_from_partials");
}

}  // namespace vae2

using namespace vae2;

extern "C" {

int64_t vae2_bn_partial_rows(const vae2_act* xd) {
  int64_t P = act_pixels(xd);
  return ceil_div(P, pix_per_block(P, xd->c));
}

int vae2_bn_stats(const float* x, const vae2_act* xd, float* partials,
                  void* stream) {
  const char* fn = "vae2_bn_stats";
  VAE2_REQUIRE(x && partials && act_ok(xd), fn, "bad arguments");
  int64_t P = act_pixels(xd);
  int64_t ppb = pix_per_block(P, xd->c);
  Act a = to_act(xd);
  if (quad_ok(xd->c) && v4_ok(x, xd->ps)) {
    VAE2_LAUNCH((chan_partials_q_kernel<0>), dim3((unsigned)ceil_div(P, ppb)), dim3(256),
                       0, as_stream(stream), x, a, (const float*)nullptr, a,
                       (const float*)nullptr, a, (const float*)nullptr, 0, ppb,
                       quad_rows(xd->c), partials);
    return check_launch(fn);
  }
  VAE2_LAUNCH((chan_partials_kernel<0>), dim3((unsigned)ceil_div(P, ppb)),
                     dim3(256), 0, as_stream(stream), x, a, (const float*)nullptr, a,
                     (const float*)nullptr, a, (const float*)nullptr, 0, ppb, partials);
  return check_launch(fn);
}

int vae2_bn_partials_reduce(const float* partials, int64_t rows, int64_t c,
                            double* sums, int accumulate, void* stream) {
  const char* fn = "vae2_bn_partials_reduce";
  VAE2_REQUIRE(partials && sums && rows > 0 && c > 0, fn, "bad arguments");
  VAE2_LAUNCH(partials_reduce_kernel, dim3((unsigned)c), dim3(256), 0,
                     as_stream(stream), partials, rows, c, sums, accumulate);
  return check_launch(fn);
}

int vae2_bn_finalize(const double* sums, double count, const float* gamma,
                     const float* beta, float* running_mean, float* running_var,
                     int64_t* num_batches_tracked, float momentum, float eps,
                     int64_t c, float* save, void* stream) {
  const char* fn = "vae2_bn_finalize";
  VAE2_REQUIRE(sums && save && c > 0 && count > 0, fn, "bad arguments");
  VAE2_REQUIRE((running_mean == nullptr) == (running_var == nullptr), fn,
               "running_mean and running_var must both be set or both be null");
  VAE2_LAUNCH(bn_finalize_kernel, dim3((unsigned)ceil_div(c, 256)), dim3(256), 0,
                     as_stream(stream), sums, count, gamma, beta, running_mean,
                     running_var, num_batches_tracked, momentum, eps, c, save);
  return check_launch(fn);
}

int vae2_bn_reduce_finalize(const float* partials, int64_t rows, int64_t c,
                            double* sums, double count, const float* gamma,
                            const float* beta, float* running_mean, float* running_var,
                            int64_t* num_batches_tracked, float momentum, float eps,
                            float* save, void* stream) {
  const char* fn = "vae2_bn_reduce_finalize";
  VAE2_REQUIRE(partials && sums && save && rows > 0 && c > 0 && count > 0, fn, "bad arguments");
  VAE2_REQUIRE((running_mean == nullptr) == (running_var == nullptr), fn,
               "running_mean and running_var must both be set or both be null");
  VAE2_LAUNCH((reduce_then_kernel<0>), dim3((unsigned)c), dim3(256), 0, as_stream(stream),
                     partials, rows, c, sums, count, gamma, beta, running_mean, running_var,
                     num_batches_tracked, momentum, eps, save, (float*)nullptr, (float*)nullptr);
  return check_launch(fn);
}

int vae2_bn_reduce_finalize_shifted(const float* partials, int64_t rows, int64_t c,
                                    double* sums, double count, const float* mean_shift,
                                    const float* gamma, const float* beta,
                                    float* running_mean, float* running_var,
                                    int64_t* num_batches_tracked, float momentum, float eps,
                                    float* save, void* stream) {
  const char* fn = "vae2_bn_reduce_finalize_shifted";
  VAE2_REQUIRE(partials && sums && save && rows > 0 && c > 0 && count > 0, fn, "bad arguments");
  VAE2_REQUIRE((running_mean == nullptr) == (running_var == nullptr), fn,
               "running_mean and running_var must both be set or both be null");
  VAE2_LAUNCH((reduce_then_kernel<0>), dim3((unsigned)c), dim3(256), 0, as_stream(stream),
              partials, rows, c, sums, count, gamma, beta, running_mean, running_var,
              num_batches_tracked, momentum, eps, save, (float*)nullptr, (float*)nullptr,
              mean_shift);
  return check_launch(fn);
}

int vae2_bn_finalize_shifted(const double* sums, double count, const float* mean_shift,
                             const float* gamma, const float* beta, float* running_mean,
                             float* running_var, int64_t* num_batches_tracked, float momentum,
                             float eps, int64_t c, float* save, void* stream) {
  const char* fn = "vae2_bn_finalize_shifted";
  VAE2_REQUIRE(sums && save && c > 0 && count > 0, fn, "bad arguments");
  VAE2_REQUIRE((running_mean == nullptr) == (running_var == nullptr), fn,
               "running_mean and running_var must both be set or both be null");
  VAE2_LAUNCH(bn_finalize_kernel, dim3((unsigned)ceil_div(c, 256)), dim3(256), 0,
              as_stream(stream), sums, count, gamma, beta, running_mean, running_var,
              num_batches_tracked, momentum, eps, c, save, mean_shift);
  return check_launch(fn);
}

int vae2_bn_bwd_reduce_param_grads(const float* partials, int64_t rows, int64_t c,
                                   double* sums, float* dgamma, float* dbeta, void* stream) {
  const char* fn = "vae2_bn_bwd_reduce_param_grads";
  VAE2_REQUIRE(partials && sums && rows > 0 && c > 0, fn, "bad arguments");
  VAE2_LAUNCH((reduce_then_kernel<1>), dim3((unsigned)c), dim3(256), 0, as_stream(stream),
                     partials, rows, c, sums, 1.0, (const float*)nullptr, (const float*)nullptr,
                     (float*)nullptr, (float*)nullptr, (int64_t*)nullptr, 0.f, 0.f, (float*)nullptr,
                     dgamma, dbeta);
  return check_launch(fn);
}

int vae2_bn_eval_coeffs(const float* gamma, const float* beta,
                        const float* running_mean, const float* running_var,
                        float eps, int64_t c, float* save, void* stream) {
  const char* fn = "vae2_bn_eval_coeffs";
  VAE2_REQUIRE(running_mean && running_var && save && c > 0, fn, "bad arguments");
  VAE2_LAUNCH(bn_eval_kernel, dim3((unsigned)ceil_div(c, 256)), dim3(256), 0,
                     as_stream(stream), gamma, beta, running_mean, running_var, eps, c,
                     save);
  return check_launch(fn);
}

int vae2_bn_apply(const float* x, const vae2_act* xd, const float* save,
                  const float* res, const vae2_act* rd, float* y,
                  const vae2_act* yd, int relu, void* stream) {
  const char* fn = "vae2_bn_apply";
  VAE2_REQUIRE(x && save && y && act_ok(xd) && act_ok(yd), fn, "bad arguments");
  VAE2_REQUIRE(xd->n == yd->n && xd->h == yd->h && xd->w == yd->w && xd->c == yd->c, fn,
               "x / y shape mismatch");
  Act r = to_act(yd);
  if (res) {
    VAE2_REQUIRE(act_ok(rd) && rd->c == xd->c && rd->h == xd->h && rd->w == xd->w, fn,
                 "residual shape mismatch");
    r = to_act(rd);
  }
  int64_t total = act_elems(xd);
  VAE2_REQUIRE(total < (int64_t(1) << 31), fn, "tensor too large");
  if (quad_ok(xd->c) && v4_ok(x, xd->ps) && v4_ok(y, yd->ps) && (!res || v4_ok(res, rd->ps))) {
    const int rows = quad_rows(xd->c);
    VAE2_LAUNCH(bn_apply_q_kernel,
                       dim3((unsigned)ceil_div(act_pixels(xd), (int64_t)rows * kApplyU)),
                       dim3(256), 0, as_stream(stream), x, to_act(xd), save, res, r, y,
                       to_act(yd), relu, rows);
    return check_launch(fn);
  }
  bool vec = (xd->c % 4 == 0) && v4_ok(x, xd->ps) && v4_ok(y, yd->ps) &&
             (!res || v4_ok(res, rd->ps)) && v4_ok(save, 4);
  if (vec) {
    VAE2_LAUNCH(bn_apply_kernel_v4, dim3(ew_blocks(total / 4)), dim3(256), 0,
                       as_stream(stream), x, to_act(xd), save, res, r, y, to_act(yd), relu,
                       FastDiv((uint32_t)(xd->c / 4)));
  } else {
    VAE2_LAUNCH(bn_apply_kernel, dim3(ew_blocks(total)), dim3(256), 0,
                       as_stream(stream), x, to_act(xd), save, res, r, y, to_act(yd), relu,
                       FastDiv((uint32_t)xd->c));
  }
  return check_launch(fn);
}

int vae2_bn_relu_bwd_reduce(const float* dy, const vae2_act* dyd,
                            const float* y, const vae2_act* yd, const float* x,
                            const vae2_act* xd, const float* save, int relu,
                            float* partials, void* stream) {
  const char* fn = "vae2_bn_relu_bwd_reduce";
  VAE2_REQUIRE(dy && x && save && partials && act_ok(dyd) && act_ok(xd), fn, "bad arguments");
  VAE2_REQUIRE(!y || act_ok(yd), fn, "bad y descriptor");
  int64_t P = act_pixels(xd);
  int64_t ppb = pix_per_block(P, xd->c);
  Act ya = (relu && y) ? to_act(yd) : to_act(xd);
  if (!relu) y = nullptr;
  if (quad_ok(xd->c) && v4_ok(x, xd->ps) && v4_ok(dy, dyd->ps) && (!y || v4_ok(y, yd->ps))) {
    VAE2_LAUNCH((chan_partials_q_kernel<1>), dim3((unsigned)ceil_div(P, ppb)), dim3(256),
                       0, as_stream(stream), x, to_act(xd), dy, to_act(dyd), y, ya, save, relu,
                       ppb, quad_rows(xd->c), partials);
    return check_launch(fn);
  }
  VAE2_LAUNCH((chan_partials_kernel<1>), dim3((unsigned)ceil_div(P, ppb)),
                     dim3(256), 0, as_stream(stream), x, to_act(xd), dy, to_act(dyd), y,
                     ya, save, relu, ppb, partials);
  return check_launch(fn);
}

int vae2_bn_bwd_param_grads(const double* sums, int64_t c, float* dgamma,
                            float* dbeta, void* stream) {
  const char* fn = "vae2_bn_bwd_param_grads";
  VAE2_REQUIRE(sums && c > 0, fn, "bad arguments");
  VAE2_LAUNCH(bn_param_grad_kernel, dim3((unsigned)ceil_div(c, 256)), dim3(256), 0,
                     as_stream(stream), sums, c, dgamma, dbeta);
  return check_launch(fn);
}

int vae2_bn_relu_bwd_apply(const float* dy, const vae2_act* dyd, const float* y,
                           const vae2_act* yd, const float* x,
                           const vae2_act* xd, const float* save,
                           const float* gamma, const double* sums, double count,
                           int relu, float* dx, const vae2_act* dxd,
                           float* dres, const vae2_act* dresd, void* stream) {
  const char* fn = "vae2_bn_relu_bwd_apply";
  VAE2_REQUIRE(dy && x && save && sums && dx && act_ok(dyd) && act_ok(xd) && act_ok(dxd),
               fn, "bad arguments");
  VAE2_REQUIRE(!y || act_ok(yd), fn, "bad y descriptor");
  VAE2_REQUIRE(!dres || act_ok(dresd), fn, "bad dres descriptor");
  int64_t total = act_elems(xd);
  VAE2_REQUIRE(total < (int64_t(1) << 31), fn, "tensor too large");
  Act ya = (relu && y) ? to_act(yd) : to_act(xd);
  if (!relu) y = nullptr;
  if (quad_ok(xd->c) && v4_ok(x, xd->ps) && v4_ok(dy, dyd->ps) && v4_ok(dx, dxd->ps) &&
      (!y || v4_ok(y, yd->ps)) && (!dres || v4_ok(dres, dresd->ps))) {
    const int rows = quad_rows(xd->c);
    VAE2_LAUNCH(bn_bwd_apply_q_kernel,
                       dim3((unsigned)ceil_div(act_pixels(xd), (int64_t)rows * kApplyU)),
                       dim3(256), 0, as_stream(stream), dy, to_act(dyd), y, ya, x, to_act(xd),
                       save, gamma, sums, count, relu, dx, to_act(dxd), dres,
                       dres ? to_act(dresd) : to_act(xd), rows);
    return check_launch(fn);
  }
  Act ra = dres ? to_act(dresd) : to_act(xd);
  VAE2_LAUNCH(bn_bwd_apply_kernel, dim3(ew_blocks(total)), dim3(256), 0,
                     as_stream(stream), dy, to_act(dyd), y, ya, x, to_act(xd), save, gamma,
                     sums, count, relu, dx, to_act(dxd), dres, ra,
                     FastDiv((uint32_t)xd->c));
  return check_launch(fn);
}

// ------------------------------------------------- multi-layer launchers ----
static bool bn_layer_quad_ok(const vae2_bn_layer& l, bool bwd) {
  const vae2_act& x = l.xd;
  if (!l.x || !l.o || !l.save || !act_ok(&x) || !quad_ok(x.c) || !v4_ok(l.x, x.ps)) return false;
  if (!v4_ok(l.o, l.od.ps) || l.od.n != x.n || l.od.h != x.h || l.od.w != x.w || l.od.c != x.c)
    return false;
  if (l.a && (!v4_ok(l.a, l.ad.ps) || l.ad.n != x.n || l.ad.h != x.h || l.ad.w != x.w ||
              l.ad.c < x.c))
    return false;
  if (bwd) {
    if (!l.dy || !v4_ok(l.dy, l.dyd.ps) || l.dyd.n != x.n || l.dyd.h != x.h || l.dyd.w != x.w)
      return false;
    if (l.dres && (!v4_ok(l.dres, l.dresd.ps) || l.dresd.c != x.c)) return false;
  }
  if (l.rx) {  // the residual BN's input (and its gradient): same pixels and channels
    const vae2_act& r = l.rxd;
    if (!l.rsave || !v4_ok(l.rx, r.ps) || r.n != x.n || r.h != x.h || r.w != x.w || r.c != x.c)
      return false;
    if (!bwd && l.a) return false;  // one residual: stored (a) or through its BN (rx)
    if (bwd && (l.dres || !l.rdx || !v4_ok(l.rdx, l.rdxd.ps) || l.rdxd.c != x.c ||
                l.rdxd.n != x.n || l.rdxd.h != x.h || l.rdxd.w != x.w))
      return false;
  }
  return act_pixels(&x) * x.c < (int64_t(1) << 31);
}

// kind 0: forward apply, 1: backward reduce, 2: backward apply
static int bn_multi_launch(int n, const vae2_bn_layer* ls, int kind, void* stream,
                           const char* fn) {
  VAE2_REQUIRE(n >= 0 && (n == 0 || ls), fn, "bad arguments");
  for (int i0 = 0; i0 < n; i0 += kBnMaxLayers) {
    BnMulti m{};
    m.n = n - i0 < kBnMaxLayers ? n - i0 : kBnMaxLayers;
    int blocks = 0;
    for (int j = 0; j < m.n; ++j) {
      const vae2_bn_layer& l = ls[i0 + j];
      VAE2_REQUIRE(bn_layer_quad_ok(l, kind != 0), fn,
                   "layer tensors must be 16-byte aligned NHWC with pixel strides % 4 == 0, "
                   "matching shapes, C <= 1024");
      VAE2_REQUIRE(kind == 0 || (kind == 1 ? l.partials != nullptr : l.sums != nullptr), fn,
                   "missing partials / sums");
      VAE2_REQUIRE(!l.rx || kind == 0 || (kind == 1 ? l.rpartials != nullptr : l.rsums != nullptr),
                   fn, "missing the residual BatchNorm's partials / sums");
      VAE2_REQUIRE(kind != 2 || l.countp || l.count > 0, fn, "bad count");
      BnLayer& L = m.L[j];
      L.x = l.x; L.a = l.a; L.o = l.o; L.dy = l.dy; L.dres = l.dres; L.part = l.partials;
      L.save = l.save; L.gamma = l.gamma; L.sums = l.sums; L.countp = l.countp;
      L.count = l.count;
      L.P = act_pixels(&l.xd);
      L.C = (int)l.xd.c;
      L.x_ps = (int)l.xd.ps; L.a_ps = (int)l.ad.ps; L.o_ps = (int)l.od.ps;
      L.dy_ps = (int)l.dyd.ps; L.dres_ps = (int)l.dresd.ps;
      L.dres_acc = l.dres_acc;
      L.relu = l.relu;
      L.rx = l.rx; L.rsave = l.rsave; L.rgamma = l.rgamma; L.rpart = l.rpartials;
      L.rsums = l.rsums; L.rdx = l.rdx;
      L.rx_ps = (int)l.rxd.ps; L.rdx_ps = (int)l.rdxd.ps;
      L.mk = l.mask;
      L.rows = quad_rows(l.xd.c);
      L.blk0 = blocks;
      if (kind == 1) {
        L.ppb = pix_per_block(L.P, L.C);
        blocks += (int)ceil_div(L.P, L.ppb);
      } else {
        blocks += (int)ceil_div(L.P, (int64_t)L.rows * kApplyU);
      }
    }
    if (blocks == 0) continue;
    m.v2 = g_bn_v2;
    m.total = blocks;
    for (int j = 0; j < m.n; ++j) {  // 32-bit buffer offsets: every extent below 2 GB
      const vae2_bn_layer& l = ls[i0 + j];
      const int64_t P = act_pixels(&l.xd);
      const int64_t ext = P * std::max({l.xd.ps, l.od.ps, l.dyd.ps, l.ad.ps, l.dresd.ps,
                                        l.rxd.ps, l.rdxd.ps, (int64_t)1}) * 4;
      if (ext >= (int64_t(1) << 31)) m.v2 = 0;
    }
    hipStream_t st = as_stream(stream);
    if (kind != 1 && m.v2 && g_bn_apply_res > 0 && blocks > g_bn_apply_res) {
      const int rounds = (blocks + g_bn_apply_res - 1) / g_bn_apply_res;
      blocks = (blocks + rounds - 1) / rounds;  // (m.total keeps the chunk count)
    }
    if (kind == 0 && m.v2)
      VAE2_LAUNCH(bn_apply_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, st, m);
    else if (kind == 0)
      VAE2_LAUNCH(bn_apply_multi_r4_kernel, dim3((unsigned)blocks), dim3(256), 0, st, m);
    else if (kind == 1 && m.v2)
      bwd_reduce_launch(m, (unsigned)blocks, st);
    else if (kind == 1)
      VAE2_LAUNCH(bn_bwd_reduce_multi_r4_kernel, dim3((unsigned)blocks), dim3(256), 0, st, m);
    else if (m.v2)
      bwd_apply_launch(m, (unsigned)blocks, st);
    else
      VAE2_LAUNCH(bn_bwd_apply_multi_r4_kernel, dim3((unsigned)blocks), dim3(256), 0, st, m);
    const int rc = check_launch(fn);
    if (rc) return rc;
  }
  return 0;
}

int vae2_bn_multi_apply(int n, const vae2_bn_layer* layers, void* stream) {
  return bn_multi_launch(n, layers, 0, stream, "vae2_bn_multi_apply");
}

int vae2_bn_multi_bwd_reduce(int n, const vae2_bn_layer* layers, void* stream) {
  return bn_multi_launch(n, layers, 1, stream, "vae2_bn_multi_bwd_reduce");
}

int vae2_bn_multi_bwd_apply(int n, const vae2_bn_layer* layers, void* stream) {
  return bn_multi_launch(n, layers, 2, stream, "vae2_bn_multi_bwd_apply");
}

static int bn_fin_pack(int n, const vae2_bn_fin* fs, int i0, FinMulti& m, int& blocks,
                       bool per_channel, const char* fn) {
  m = FinMulti{};
  m.n = n - i0 < kBnMaxLayers ? n - i0 : kBnMaxLayers;
  blocks = 0;
  for (int j = 0; j < m.n; ++j) {
    const vae2_bn_fin& f = fs[i0 + j];
    VAE2_REQUIRE(f.sums && f.c > 0 && f.c <= (1 << 20), fn, "bad layer");
    FinLayer& L = m.L[j];
    L.part = f.partials; L.sums = f.sums; L.gamma = f.gamma; L.beta = f.beta;
    L.rmean = f.running_mean; L.rvar = f.running_var; L.nbt = f.num_batches_tracked;
    L.save = f.save; L.dgamma = f.dgamma; L.dbeta = f.dbeta; L.countp = f.countp;
    L.count = f.count; L.rows = f.rows; L.momentum = f.momentum; L.eps = f.eps;
    L.C = (int)f.c;
    L.blk0 = blocks;
    blocks += per_channel ? (int)f.c : 1;
  }
  return 0;
}

int vae2_bn_multi_reduce(int n, const vae2_bn_fin* fins, int mode, void* stream) {
  const char* fn = "vae2_bn_multi_reduce";
  VAE2_REQUIRE(n >= 0 && (n == 0 || fins) && mode >= 0 && mode <= 2, fn, "bad arguments");
  for (int i = 0; i < n; ++i) {
    const vae2_bn_fin& f = fins[i];
    VAE2_REQUIRE(f.partials && f.rows > 0, fn, "missing partials");
    VAE2_REQUIRE(mode != 0 || (f.save && (f.countp || f.count > 0)), fn, "missing save / count");
    VAE2_REQUIRE((f.running_mean == nullptr) == (f.running_var == nullptr), fn,
                 "running_mean and running_var must both be set or both be null");
  }
  for (int i0 = 0; i0 < n; i0 += kBnMaxLayers) {
    FinMulti m;
    int blocks;
    int rc = bn_fin_pack(n, fins, i0, m, blocks, true, fn);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    if (mode == 0)
      VAE2_LAUNCH(reduce_then_multi_kernel<0>, dim3((unsigned)blocks), dim3(256), 0, st, m);
    else if (mode == 1)
      VAE2_LAUNCH(reduce_then_multi_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, st, m);
    else
      VAE2_LAUNCH(reduce_then_multi_kernel<2>, dim3((unsigned)blocks), dim3(256), 0, st, m);
    rc = check_launch(fn);
    if (rc) return rc;
  }
  return 0;
}

int vae2_bn_multi_finalize(int n, const vae2_bn_fin* fins, void* stream) {
  const char* fn = "vae2_bn_multi_finalize";
  VAE2_REQUIRE(n >= 0 && (n == 0 || fins), fn, "bad arguments");
  for (int i = 0; i < n; ++i)
    VAE2_REQUIRE(fins[i].save && (fins[i].countp || fins[i].count > 0), fn,
                 "missing save / count");
  for (int i0 = 0; i0 < n; i0 += kBnMaxLayers) {
    FinMulti m;
    int blocks;
    int rc = bn_fin_pack(n, fins, i0, m, blocks, false, fn);
    if (rc) return rc;
    VAE2_LAUNCH(bn_finalize_multi_kernel, dim3((unsigned)m.n), dim3(256), 0, as_stream(stream), m);
    rc = check_launch(fn);
    if (rc) return rc;
  }
  return 0;
}

}  // extern "C"
