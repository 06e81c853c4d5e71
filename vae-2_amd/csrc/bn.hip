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
#include "common.h"

namespace vae2 {

// ---------------------------------------------------- partial reductions ----
// Pixels per block for per-channel reductions.
static int64_t pix_per_block(int64_t P) {
  int64_t ppb = ceil_div(P, 1024);
  if (ppb < 32) ppb = 32;
  return ppb;
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
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }

__device__ __forceinline__ f4 chan4(const float* a, int c, int C) {
  f4 v;
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = (c + k < C) ? a[c + k] : 0.f;
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

static inline int quad_rows(int64_t C) { return 256 / (int)((C + 3) / 4); }
constexpr int kApplyU = 4;  // pixels per thread in the apply kernels

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

// One block per channel: sums[q][c] (+)= sum_rows part[q][row][c] in double.
__global__ __launch_bounds__(256) void partials_reduce_kernel(
    const float* __restrict__ part, int64_t rows, int64_t C, double* sums,
    int accumulate) {
  __shared__ double red[2][4];
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  double a = 0.0, b = 0.0;
  for (int64_t r = tid; r < rows; r += 256) {
    a += (double)part[r * C + c];
    b += (double)part[(rows + r) * C + c];
  }
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
__global__ __launch_bounds__(256) void reduce_then_kernel(
    const float* __restrict__ part, int64_t rows, int64_t C, double* sums, double count,
    const float* gamma, const float* beta, float* rmean, float* rvar, int64_t* nbt,
    float momentum, float eps, float* save, float* dgamma, float* dbeta) {
  __shared__ double red[2][4];
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  double a = 0.0, b = 0.0;
  for (int64_t r = tid; r < rows; r += 256) {
    a += (double)part[r * C + c];
    b += (double)part[(rows + r) * C + c];
  }
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
  const double mean = s0 / count;
  double var = s1 / count - mean * mean;
  if (var < 0.0) var = 0.0;
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
                                   float* save) {
  int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (c == 0 && nbt) nbt[0] += 1;
  if (c >= C) return;
  double mean = sums[c] / count;
  double var = sums[C + c] / count - mean * mean;
  if (var < 0.0) var = 0.0;
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
  for (int64_t r = tid; r < rows; r += 256) a += (double)part[r * C + c];
  a = wave_sum_d(a);
  if ((tid & 63) == 0) red[tid >> 6] = a;
  __syncthreads();
  if (tid == 0) {
    float s = (float)(red[0] + red[1] + red[2] + red[3]);
    out[c] = accumulate ? out[c] + s : s;
  }
}

static bool v4_ok(const void* p, int64_t ps) {
  return ((uintptr_t)p % 16 == 0) && (ps % 4 == 0);
}

static bool quad_ok(int64_t c) { return (c + 3) / 4 <= 256; }

int bias_grad_from_partials(const float* partials, int64_t rows, int64_t c,
                            float* dbias, int accumulate, void* stream) {
  hipLaunchKernelGGL(colsum_to_float_kernel, dim3((unsigned)c), dim3(256), 0,
                     as_stream(stream), partials, rows, c, dbias, accumulate);
  return check_launch("bias_grad_from_partials");
}

}  // namespace vae2

using namespace vae2;

extern "C" {

int64_t vae2_bn_partial_rows(const vae2_act* xd) {
  int64_t P = act_pixels(xd);
  return ceil_div(P, pix_per_block(P));
}

int vae2_bn_stats(const float* x, const vae2_act* xd, float* partials,
                  void* stream) {
  const char* fn = "vae2_bn_stats";
  VAE2_REQUIRE(x && partials && act_ok(xd), fn, "bad arguments");
  int64_t P = act_pixels(xd);
  int64_t ppb = pix_per_block(P);
  Act a = to_act(xd);
  if (quad_ok(xd->c) && v4_ok(x, xd->ps)) {
    hipLaunchKernelGGL((chan_partials_q_kernel<0>), dim3((unsigned)ceil_div(P, ppb)), dim3(256),
                       0, as_stream(stream), x, a, (const float*)nullptr, a,
                       (const float*)nullptr, a, (const float*)nullptr, 0, ppb,
                       quad_rows(xd->c), partials);
    return check_launch(fn);
  }
  hipLaunchKernelGGL((chan_partials_kernel<0>), dim3((unsigned)ceil_div(P, ppb)),
                     dim3(256), 0, as_stream(stream), x, a, (const float*)nullptr, a,
                     (const float*)nullptr, a, (const float*)nullptr, 0, ppb, partials);
  return check_launch(fn);
}

int vae2_bn_partials_reduce(const float* partials, int64_t rows, int64_t c,
                            double* sums, int accumulate, void* stream) {
  const char* fn = "vae2_bn_partials_reduce";
  VAE2_REQUIRE(partials && sums && rows > 0 && c > 0, fn, "bad arguments");
  hipLaunchKernelGGL(partials_reduce_kernel, dim3((unsigned)c), dim3(256), 0,
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
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((unsigned)ceil_div(c, 256)), dim3(256), 0,
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
  hipLaunchKernelGGL((reduce_then_kernel<0>), dim3((unsigned)c), dim3(256), 0, as_stream(stream),
                     partials, rows, c, sums, count, gamma, beta, running_mean, running_var,
                     num_batches_tracked, momentum, eps, save, (float*)nullptr, (float*)nullptr);
  return check_launch(fn);
}

int vae2_bn_bwd_reduce_param_grads(const float* partials, int64_t rows, int64_t c,
                                   double* sums, float* dgamma, float* dbeta, void* stream) {
  const char* fn = "vae2_bn_bwd_reduce_param_grads";
  VAE2_REQUIRE(partials && sums && rows > 0 && c > 0, fn, "bad arguments");
  hipLaunchKernelGGL((reduce_then_kernel<1>), dim3((unsigned)c), dim3(256), 0, as_stream(stream),
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
  hipLaunchKernelGGL(bn_eval_kernel, dim3((unsigned)ceil_div(c, 256)), dim3(256), 0,
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
    hipLaunchKernelGGL(bn_apply_q_kernel,
                       dim3((unsigned)ceil_div(act_pixels(xd), (int64_t)rows * kApplyU)),
                       dim3(256), 0, as_stream(stream), x, to_act(xd), save, res, r, y,
                       to_act(yd), relu, rows);
    return check_launch(fn);
  }
  bool vec = (xd->c % 4 == 0) && v4_ok(x, xd->ps) && v4_ok(y, yd->ps) &&
             (!res || v4_ok(res, rd->ps)) && v4_ok(save, 4);
  if (vec) {
    hipLaunchKernelGGL(bn_apply_kernel_v4, dim3(ew_blocks(total / 4)), dim3(256), 0,
                       as_stream(stream), x, to_act(xd), save, res, r, y, to_act(yd), relu,
                       FastDiv((uint32_t)(xd->c / 4)));
  } else {
    hipLaunchKernelGGL(bn_apply_kernel, dim3(ew_blocks(total)), dim3(256), 0,
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
  int64_t ppb = pix_per_block(P);
  Act ya = (relu && y) ? to_act(yd) : to_act(xd);
  if (!relu) y = nullptr;
  if (quad_ok(xd->c) && v4_ok(x, xd->ps) && v4_ok(dy, dyd->ps) && (!y || v4_ok(y, yd->ps))) {
    hipLaunchKernelGGL((chan_partials_q_kernel<1>), dim3((unsigned)ceil_div(P, ppb)), dim3(256),
                       0, as_stream(stream), x, to_act(xd), dy, to_act(dyd), y, ya, save, relu,
                       ppb, quad_rows(xd->c), partials);
    return check_launch(fn);
  }
  hipLaunchKernelGGL((chan_partials_kernel<1>), dim3((unsigned)ceil_div(P, ppb)),
                     dim3(256), 0, as_stream(stream), x, to_act(xd), dy, to_act(dyd), y,
                     ya, save, relu, ppb, partials);
  return check_launch(fn);
}

int vae2_bn_bwd_param_grads(const double* sums, int64_t c, float* dgamma,
                            float* dbeta, void* stream) {
  const char* fn = "vae2_bn_bwd_param_grads";
  VAE2_REQUIRE(sums && c > 0, fn, "bad arguments");
  hipLaunchKernelGGL(bn_param_grad_kernel, dim3((unsigned)ceil_div(c, 256)), dim3(256), 0,
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
    hipLaunchKernelGGL(bn_bwd_apply_q_kernel,
                       dim3((unsigned)ceil_div(act_pixels(xd), (int64_t)rows * kApplyU)),
                       dim3(256), 0, as_stream(stream), dy, to_act(dyd), y, ya, x, to_act(xd),
                       save, gamma, sums, count, relu, dx, to_act(dxd), dres,
                       dres ? to_act(dresd) : to_act(xd), rows);
    return check_launch(fn);
  }
  Act ra = dres ? to_act(dresd) : to_act(xd);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(ew_blocks(total)), dim3(256), 0,
                     as_stream(stream), dy, to_act(dyd), y, ya, x, to_act(xd), save, gamma,
                     sums, count, relu, dx, to_act(dxd), dres, ra,
                     FastDiv((uint32_t)xd->c));
  return check_launch(fn);
}

}  // extern "C"
