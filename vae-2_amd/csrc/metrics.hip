// Evaluation metrics of the prior-sampling inference (function.py:55-316,
// tools/inference.py): frames back to [0, 255] images, L1 / PSNR sums, SSIM and the
// per-level pieces of MS-SSIM.
//
//   _to_image (function.py:86-97): x*std + mean, *255, clip to [0, 255]
//                                   -> vae2_to_image
//   recon_loss = mean|a - b| (:252), PSNR (criterion.py:106-116) = 20 log10(255 / sqrt(mse))
//                                   -> vae2_absdiff_sqdiff_sum
//   pytorch_msssim ssim / ms_ssim (third-party, absent from the reference tree; restated
//   from pytorch_msssim 1.0.0): separable Gaussian window (valid convolution), per-channel
//   means of the SSIM and contrast-structure maps
//                                   -> vae2_ssim_partials + vae2_ssim_finish
//   F.avg_pool2d(kernel 2, padding = size % 2) between MS-SSIM levels
//                                   -> vae2_avgpool2x2
//
// Images are NCHW fp32 planes (the layout of the reference's tensors).  Every reduction
// is per-block partials in double, summed in a fixed order (deterministic).
#include "common.h"

namespace vae2 {

constexpr int kWin = 11;       // Gaussian window taps (pytorch_msssim default win_size)
constexpr int kTH = 16;        // output rows per workgroup
constexpr int kTW = 64;        // output columns per workgroup
constexpr int kIH = kTH + kWin - 1;
constexpr int kIW = kTW + kWin - 1;

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  v = wave_sum_d(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) s = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return s;  // valid in thread 0
}

// The reference's arithmetic, element by element: x (fp32) *= std (fp64 array) -> fp32;
// += mean (fp64) -> fp32; *= 255.0 in fp32; clip to [0, 255].
__global__ __launch_bounds__(256) void to_image_kernel(const float* __restrict__ x,
                                                       float* __restrict__ y, int64_t total,
                                                       uint32_t hw, uint32_t c, double m0,
                                                       double m1, double m2, double s0,
                                                       double s1, double s2) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    const uint32_t ch = (uint32_t)((i / hw) % c) % 3u;
    const double m = ch == 0 ? m0 : (ch == 1 ? m1 : m2);
    const double s = ch == 0 ? s0 : (ch == 1 ? s1 : s2);
    float v = (float)((double)x[i] * s);
    v = (float)((double)v + m);
    v = v * 255.0f;
    v = fminf(fmaxf(v, 0.f), 255.f);
    y[i] = v;
  }
}

// partials[b] = (sum |a-b|, sum (a-b)^2) over a grid-stride slice, per plane group
__global__ __launch_bounds__(256) void absdiff_sqdiff_kernel(const float* __restrict__ a,
                                                             const float* __restrict__ b,
                                                             int64_t total,
                                                             double* __restrict__ part) {
  __shared__ double red[4];
  double s1 = 0.0, s2 = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    const float d = a[i] - b[i];
    s1 += (double)fabsf(d);
    s2 += (double)(d * d);
  }
  s1 = block_sum_d(s1, red);
  s2 = block_sum_d(s2, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s1;
    part[2 * blockIdx.x + 1] = s2;
  }
}

__global__ __launch_bounds__(256) void sum_pairs_kernel(const double* __restrict__ part,
                                                        int n, double* __restrict__ out) {
  __shared__ double red[4];
  double s1 = 0.0, s2 = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    s1 += part[2 * i];
    s2 += part[2 * i + 1];
  }
  s1 = block_sum_d(s1, red);
  s2 = block_sum_d(s2, red);
  if (threadIdx.x == 0) {
    out[0] = s1;
    out[1] = s2;
  }
}

// SSIM of one (kTH x kTW) output tile of one plane (blockIdx.z = n*C + c).  Valid
// convolution: output (h - 10) x (w - 10).  Both images' halo tiles are staged in LDS,
// the five horizontally filtered maps (x, y, x^2, y^2, xy) go to LDS, then each thread
// filters its output pixels vertically and accumulates the SSIM and CS map values.
// part[(plane * tiles + tile) * 2 + {0, 1}] = (sum ssim_map, sum cs_map) of the tile.
__global__ __launch_bounds__(256) void ssim_tile_kernel(const float* __restrict__ X,
                                                        const float* __restrict__ Y, int h,
                                                        int w, const float* __restrict__ win,
                                                        float C1, float C2,
                                                        double* __restrict__ part) {
  __shared__ float sx[kIH][kIW + 1];
  __shared__ float sy[kIH][kIW + 1];
  __shared__ float hf[5][kIH][kTW + 1];
  __shared__ float g[kWin];
  __shared__ double red[4];
  const int tid = threadIdx.x;
  const int ho = h - (kWin - 1), wo = w - (kWin - 1);
  const int x0 = blockIdx.x * kTW, y0 = blockIdx.y * kTH;
  const int64_t plane = blockIdx.z;
  const float* xp = X + plane * (int64_t)h * w;
  const float* yp = Y + plane * (int64_t)h * w;
  if (tid < kWin) g[tid] = win[tid];
  for (int i = tid; i < kIH * kIW; i += 256) {
    const int r = i / kIW, col = i - r * kIW;
    const int gy = y0 + r, gx = x0 + col;
    const bool in = gy < h && gx < w;
    const int64_t off = (int64_t)gy * w + gx;
    sx[r][col] = in ? xp[off] : 0.f;
    sy[r][col] = in ? yp[off] : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < kIH * kTW; i += 256) {
    const int r = i / kTW, col = i - r * kTW;
    float a1 = 0.f, a2 = 0.f, a11 = 0.f, a22 = 0.f, a12 = 0.f;
#pragma unroll
    for (int k = 0; k < kWin; ++k) {
      const float gx = g[k], u = sx[r][col + k], v = sy[r][col + k];
      a1 = fmaf(gx, u, a1);
      a2 = fmaf(gx, v, a2);
      a11 = fmaf(gx, u * u, a11);
      a22 = fmaf(gx, v * v, a22);
      a12 = fmaf(gx, u * v, a12);
    }
    hf[0][r][col] = a1;
    hf[1][r][col] = a2;
    hf[2][r][col] = a11;
    hf[3][r][col] = a22;
    hf[4][r][col] = a12;
  }
  __syncthreads();
  double ss = 0.0, cs = 0.0;
  for (int i = tid; i < kTH * kTW; i += 256) {
    const int r = i / kTW, col = i - r * kTW;
    if (y0 + r >= ho || x0 + col >= wo) continue;
    float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
    for (int k = 0; k < kWin; ++k) {
      const float gk = g[k];
      m1 = fmaf(gk, hf[0][r + k][col], m1);
      m2 = fmaf(gk, hf[1][r + k][col], m2);
      e11 = fmaf(gk, hf[2][r + k][col], e11);
      e22 = fmaf(gk, hf[3][r + k][col], e22);
      e12 = fmaf(gk, hf[4][r + k][col], e12);
    }
    const float m1s = m1 * m1, m2s = m2 * m2, m12 = m1 * m2;
    const float s1 = e11 - m1s, s2 = e22 - m2s, s12 = e12 - m12;
    const float csv = (2.f * s12 + C2) / (s1 + s2 + C2);
    const float ssv = ((2.f * m12 + C1) / (m1s + m2s + C1)) * csv;
    ss += (double)ssv;
    cs += (double)csv;
  }
  ss = block_sum_d(ss, red);
  cs = block_sum_d(cs, red);
  if (tid == 0) {
    const int64_t t = plane * ((int64_t)gridDim.x * gridDim.y) + blockIdx.y * gridDim.x +
                      blockIdx.x;
    part[2 * t] = ss;
    part[2 * t + 1] = cs;
  }
}

// out[plane*2 + {0,1}] = (mean ssim_map, mean cs_map): one block per plane, fixed order
__global__ __launch_bounds__(256) void ssim_finish_kernel(const double* __restrict__ part,
                                                          int tiles, double inv_count,
                                                          double* __restrict__ out) {
  __shared__ double red[4];
  const double* p = part + (int64_t)blockIdx.x * tiles * 2;
  double s1 = 0.0, s2 = 0.0;
  for (int i = threadIdx.x; i < tiles; i += 256) {
    s1 += p[2 * i];
    s2 += p[2 * i + 1];
  }
  s1 = block_sum_d(s1, red);
  s2 = block_sum_d(s2, red);
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = s1 * inv_count;
    out[2 * blockIdx.x + 1] = s2 * inv_count;
  }
}

// F.avg_pool2d(kernel 2, stride 2, padding (h%2, w%2), count_include_pad=True)
__global__ __launch_bounds__(256) void avgpool2x2_kernel(const float* __restrict__ x,
                                                         float* __restrict__ y, int64_t planes,
                                                         int h, int w, int ho, int wo, int ph,
                                                         int pw) {
  const int64_t total = planes * ho * wo;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    const int64_t pl = i / ((int64_t)ho * wo);
    const int rem = (int)(i - pl * ho * wo);
    const int oy = rem / wo, ox = rem - oy * wo;
    const float* xp = x + pl * (int64_t)h * w;
    float s = 0.f;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int iy = 2 * oy - ph + dy, ix = 2 * ox - pw + dx;
        if (iy >= 0 && iy < h && ix >= 0 && ix < w) s += xp[(int64_t)iy * w + ix];
      }
    y[i] = s / 4.f;
  }
}

static unsigned grid_for(int64_t n) {
  int64_t b = ceil_div(n, 256);
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (unsigned)b;
}

}  // namespace vae2

using namespace vae2;

extern "C" {

int vae2_to_image(const float* x, float* y, int64_t n, int64_t c, int64_t h, int64_t w,
                  const double* mean3, const double* std3, void* stream) {
  const char* fn = "vae2_to_image";
  VAE2_REQUIRE(x && y && mean3 && std3 && n > 0 && c > 0 && h > 0 && w > 0, fn,
               "bad arguments");
  VAE2_REQUIRE(h * w < (int64_t(1) << 32), fn, "plane too large");
  const int64_t total = n * c * h * w;
  VAE2_LAUNCH(to_image_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), x, y,
              total, (uint32_t)(h * w), (uint32_t)c, mean3[0], mean3[1], mean3[2], std3[0],
              std3[1], std3[2]);
  return check_launch(fn);
}

int64_t vae2_metrics_ws_size(int64_t planes, int64_t h, int64_t w) {
  if (planes <= 0 || h < kWin || w < kWin) return 2 * 4096;
  const int64_t tiles = ceil_div(w - (kWin - 1), kTW) * ceil_div(h - (kWin - 1), kTH);
  const int64_t t = 2 * planes * tiles;
  return t > 2 * 4096 ? t : 2 * 4096;
}

int vae2_absdiff_sqdiff_sum(const float* a, const float* b, int64_t n, double* ws,
                            double* out, void* stream) {
  const char* fn = "vae2_absdiff_sqdiff_sum";
  VAE2_REQUIRE(a && b && ws && out && n > 0, fn, "bad arguments");
  const unsigned nb = grid_for(n);
  hipStream_t s = as_stream(stream);
  VAE2_LAUNCH(absdiff_sqdiff_kernel, dim3(nb), dim3(256), 0, s, a, b, n, ws);
  int rc = check_launch(fn);
  if (rc) return rc;
  VAE2_LAUNCH(sum_pairs_kernel, dim3(1), dim3(256), 0, s, (const double*)ws, (int)nb, out);
  return check_launch(fn);
}

int vae2_ssim(const float* x, const float* y, int64_t planes, int64_t h, int64_t w,
              const float* win, int win_size, float c1, float c2, double* ws, double* out,
              void* stream) {
  const char* fn = "vae2_ssim";
  VAE2_REQUIRE(x && y && win && ws && out && planes > 0, fn, "bad arguments");
  VAE2_REQUIRE(win_size == kWin, fn, "only the 11-tap window is supported");
  VAE2_REQUIRE(h >= kWin && w >= kWin && h * w < (int64_t(1) << 31), fn,
               "image sides must be >= the window size");
  VAE2_REQUIRE(planes < 65536, fn, "too many planes");
  const int ho = (int)h - (kWin - 1), wo = (int)w - (kWin - 1);
  const dim3 grid((unsigned)ceil_div(wo, kTW), (unsigned)ceil_div(ho, kTH), (unsigned)planes);
  hipStream_t s = as_stream(stream);
  VAE2_LAUNCH(ssim_tile_kernel, grid, dim3(256), 0, s, x, y, (int)h, (int)w, win, c1, c2, ws);
  int rc = check_launch(fn);
  if (rc) return rc;
  VAE2_LAUNCH(ssim_finish_kernel, dim3((unsigned)planes), dim3(256), 0, s, (const double*)ws,
              (int)(grid.x * grid.y), 1.0 / ((double)ho * wo), out);
  return check_launch(fn);
}

int vae2_avgpool2x2(const float* x, float* y, int64_t planes, int64_t h, int64_t w,
                    void* stream) {
  const char* fn = "vae2_avgpool2x2";
  VAE2_REQUIRE(x && y && planes > 0 && h > 0 && w > 0, fn, "bad arguments");
  const int ph = (int)(h % 2), pw = (int)(w % 2);
  const int ho = (int)((h + 2 * ph - 2) / 2 + 1), wo = (int)((w + 2 * pw - 2) / 2 + 1);
  VAE2_LAUNCH(avgpool2x2_kernel, dim3(grid_for(planes * ho * wo)), dim3(256), 0,
              as_stream(stream), x, y, planes, (int)h, (int)w, ho, wo, ph, pw);
  return check_launch(fn);
}

}  // extern "C"
