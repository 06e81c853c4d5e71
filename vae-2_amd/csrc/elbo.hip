// ELBO terms, reparameterisation sampler, anomaly check and the Adam step.
//
//   L1Loss (criterion.py:61-69)            -> vae2_l1_fwd / vae2_l1_bwd
//   KLLoss (criterion.py:72-87) + reparam
//     z = mu + exp(0.5*logvar)*eps (utils.py:85-101) -> vae2_reparam_kl_fwd / _bwd
//   loss assembly (utils.py:150-152)       -> vae2_weighted_sum
//   _anomoly_detection (utils.py:63-65)    -> vae2_nonfinite_check
//   torch.optim.Adam (train.py:251-261)    -> vae2_adam_step
//   lsgan_adversarial_loss (criterion.py:90-103): MSELoss(sum) vs ones / zeros / batch
//                                          -> vae2_lsgan_fwd / vae2_lsgan_bwd
#include "common.h"

namespace vae2 {

static unsigned reduce_blocks(int64_t n) {
  int64_t b = ceil_div(n, 256 * 4);
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return (unsigned)b;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int tid = threadIdx.x;
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  float s = 0.f;
  if (tid == 0) s = red[0] + red[1] + red[2] + red[3];
  return s;  // valid in thread 0
}

__global__ __launch_bounds__(256) void l1_partials_kernel(const float* __restrict__ p, Act pd,
                                                          const float* __restrict__ t, Act td,
                                                          float* __restrict__ ws,
                                                          FastDiv cdiv) {
  __shared__ float red[4];
  const uint32_t C = (uint32_t)pd.c;
  const uint32_t total = (uint32_t)(pd.n * pd.h * pd.w) * C;
  float s = 0.f;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t px = cdiv.div(i);
    uint32_t c = i - px * C;
    s += fabsf(p[(int64_t)px * pd.ps + c] - t[(int64_t)px * td.ps + c]);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = s;
}

// out[0] (+)= scale * sum(ws[0..n))   (single block, fixed order)
__global__ __launch_bounds__(256) void finish_sum_kernel(const float* __restrict__ ws, int n,
                                                         float scale, float* out,
                                                         int accumulate) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += (double)ws[i];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float v = (float)(red[0] + red[1] + red[2] + red[3]) * scale;
    out[0] = accumulate ? out[0] + v : v;
  }
}

__global__ __launch_bounds__(256) void l1_bwd_kernel(const float* __restrict__ p, Act pd,
                                                     const float* __restrict__ t, Act td,
                                                     const float* __restrict__ gout, float scale,
                                                     float* __restrict__ dp, Act dpd, float beta,
                                                     FastDiv cdiv) {
  const uint32_t C = (uint32_t)pd.c;
  const uint32_t total = (uint32_t)(pd.n * pd.h * pd.w) * C;
  const float g = gout[0] * scale;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t px = cdiv.div(i);
    uint32_t c = i - px * C;
    float d = p[(int64_t)px * pd.ps + c] - t[(int64_t)px * td.ps + c];
    float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    float* dst = dp + (int64_t)px * dpd.ps + c;
    float v = sg * g;
    *dst = (beta != 0.f) ? v + beta * *dst : v;
  }
}

// sum (x - target)^2 partials (target a constant: 1 for 'real', 0 for 'fake')
__global__ __launch_bounds__(256) void sqdiff_partials_kernel(const float* __restrict__ x, Act xd,
                                                              float target,
                                                              float* __restrict__ ws,
                                                              FastDiv cdiv) {
  __shared__ float red[4];
  const uint32_t C = (uint32_t)xd.c;
  const uint32_t total = (uint32_t)(xd.n * xd.h * xd.w) * C;
  float s = 0.f;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t px = cdiv.div(i);
    uint32_t c = i - px * C;
    const float d = x[(int64_t)px * xd.ps + c] - target;
    s = __builtin_fmaf(d, d, s);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = s;
}

// dx (+)= 2 * scale * gout * (x - target)
__global__ __launch_bounds__(256) void sqdiff_bwd_kernel(const float* __restrict__ x, Act xd,
                                                         float target,
                                                         const float* __restrict__ gout,
                                                         float scale, float* __restrict__ dx,
                                                         Act dxd, float beta, FastDiv cdiv) {
  const uint32_t C = (uint32_t)xd.c;
  const uint32_t total = (uint32_t)(xd.n * xd.h * xd.w) * C;
  const float g = 2.f * gout[0] * scale;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t px = cdiv.div(i);
    uint32_t c = i - px * C;
    const float v = g * (x[(int64_t)px * xd.ps + c] - target);
    float* dst = dx + (int64_t)px * dxd.ps + c;
    *dst = (beta != 0.f) ? v + beta * *dst : v;
  }
}

__global__ __launch_bounds__(256) void reparam_kl_kernel(const float* __restrict__ mv, Act md,
                                                         const float* __restrict__ eps, Act ed,
                                                         float* __restrict__ z, Act zd,
                                                         int prior, float* __restrict__ ws,
                                                         FastDiv cdiv) {
  __shared__ float red[4];
  const uint32_t Z = (uint32_t)zd.c;
  const uint32_t total = (uint32_t)(zd.n * zd.h * zd.w) * Z;
  float s = 0.f;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t px = cdiv.div(i);
    uint32_t c = i - px * Z;
    float mu = mv[(int64_t)px * md.ps + c];
    float lv = mv[(int64_t)px * md.ps + Z + c];
    float e = eps[(int64_t)px * ed.ps + c];
    z[(int64_t)px * zd.ps + c] = prior ? e : mu + expf(lv * 0.5f) * e;
    s += 0.5f * (mu * mu + expf(lv) - lv - 1.f);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void reparam_kl_bwd_kernel(
    const float* __restrict__ mv, Act md, const float* __restrict__ eps, Act ed,
    const float* __restrict__ dz, Act dzd, const float* __restrict__ gkl, float scale,
    float* __restrict__ dmv, Act dmd, FastDiv cdiv) {
  const uint32_t Z = (uint32_t)ed.c;
  const uint32_t total = (uint32_t)(ed.n * ed.h * ed.w) * Z;
  const float gk = gkl ? gkl[0] * scale : 0.f;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t px = cdiv.div(i);
    uint32_t c = i - px * Z;
    float mu = mv[(int64_t)px * md.ps + c];
    float lv = mv[(int64_t)px * md.ps + Z + c];
    float e = eps[(int64_t)px * ed.ps + c];
    float g = dz ? dz[(int64_t)px * dzd.ps + c] : 0.f;
    float dmu = g + gk * mu;
    float dlv = g * e * 0.5f * expf(lv * 0.5f) + gk * 0.5f * (expf(lv) - 1.f);
    dmv[(int64_t)px * dmd.ps + c] = dmu;
    dmv[(int64_t)px * dmd.ps + Z + c] = dlv;
  }
}

struct WSum {
  const float* t[8];
  float l[8];
  int n;
};

__global__ void weighted_sum_kernel(WSum w, float* total) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float s = 0.f;
  for (int i = 0; i < w.n; ++i) s += w.l[i] * w.t[i][0];
  total[0] = s;
}

__global__ __launch_bounds__(256) void nonfinite_kernel(const float* __restrict__ x, int64_t n,
                                                        int32_t* flag) {
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v = x[i];
    bad |= !isfinite(v);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p,
                                                   const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   int64_t n, float lr_corr, float b1,
                                                   float b2, float eps, float wd,
                                                   float bc2_sqrt) {
  const float w1 = 1.f - b1;
  const float w2 = 1.f - b2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i];
    float pi = p[i];
    if (wd != 0.f) gi = gi + wd * pi;
    float mi = m[i];
    mi = mi + w1 * (gi - mi);  // lerp(m, g, 1 - b1), weight < 0.5 branch
    float vi = v[i] * b2 + w2 * (gi * gi);
    float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = pi + (-lr_corr) * (mi / denom);
    m[i] = mi;
    v[i] = vi;
  }
}

// Device-resident step counter for graph replay: state = {step, lr} (double),
// coeffs = {lr / (1 - b1^step), sqrt(1 - b2^step)} (float), as vae2_adam_step's host math.
__global__ void adam_coeffs_kernel(double* state, float b1, float b2, float* coeffs) {
  const double step = state[0] + 1.0;
  state[0] = step;
  const double lr = (double)(float)state[1];
  coeffs[0] = (float)(lr / (1.0 - pow((double)b1, step)));
  coeffs[1] = (float)sqrt(1.0 - pow((double)b2, step));
}

__global__ __launch_bounds__(256) void adam_dev_kernel(float* __restrict__ p,
                                                       const float* __restrict__ g,
                                                       float* __restrict__ m,
                                                       float* __restrict__ v, int64_t n,
                                                       const float* __restrict__ coeffs,
                                                       float b1, float b2, float eps, float wd) {
  const float lr_corr = coeffs[0];
  const float bc2_sqrt = coeffs[1];
  const float w1 = 1.f - b1;
  const float w2 = 1.f - b2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i];
    float pi = p[i];
    if (wd != 0.f) gi = gi + wd * pi;
    float mi = m[i];
    mi = mi + w1 * (gi - mi);
    float vi = v[i] * b2 + w2 * (gi * gi);
    float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = pi + (-lr_corr) * (mi / denom);
    m[i] = mi;
    v[i] = vi;
  }
}

__global__ void scale_kernel(float* dst, const float* src, int64_t n, float s) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i] * s;
}

}  // namespace vae2

using namespace vae2;

extern "C" {

int64_t vae2_reduce_ws_size(int64_t n) { return reduce_blocks(n); }

int vae2_l1_fwd(const float* p, const vae2_act* pd, const float* t,
                const vae2_act* td, float scale, float* ws, float* out,
                void* stream) {
  const char* fn = "vae2_l1_fwd";
  VAE2_REQUIRE(p && t && ws && out && act_ok(pd) && act_ok(td), fn, "bad arguments");
  VAE2_REQUIRE(pd->n == td->n && pd->h == td->h && pd->w == td->w && pd->c == td->c, fn,
               "predict / target shape mismatch");
  int64_t total = act_elems(pd);
  unsigned nb = reduce_blocks(total);
  hipStream_t s = as_stream(stream);
  VAE2_LAUNCH(l1_partials_kernel, dim3(nb), dim3(256), 0, s, p, to_act(pd), t,
                     to_act(td), ws, FastDiv((uint32_t)pd->c));
  int rc = check_launch(fn);
  if (rc) return rc;
  VAE2_LAUNCH(finish_sum_kernel, dim3(1), dim3(256), 0, s, (const float*)ws, (int)nb,
                     scale, out, 0);
  return check_launch(fn);
}

int vae2_l1_bwd(const float* p, const vae2_act* pd, const float* t,
                const vae2_act* td, const float* gout, float scale, float* dp,
                const vae2_act* dpd, float beta, void* stream) {
  const char* fn = "vae2_l1_bwd";
  VAE2_REQUIRE(p && t && gout && dp && act_ok(pd) && act_ok(td) && act_ok(dpd), fn,
               "bad arguments");
  int64_t total = act_elems(pd);
  VAE2_LAUNCH(l1_bwd_kernel, dim3(ew_blocks(total)), dim3(256), 0, as_stream(stream), p,
                     to_act(pd), t, to_act(td), gout, scale, dp, to_act(dpd), beta,
                     FastDiv((uint32_t)pd->c));
  return check_launch(fn);
}

int vae2_lsgan_fwd(const float* x, const vae2_act* xd, float target, float scale, float* ws,
                   float* out, void* stream) {
  const char* fn = "vae2_lsgan_fwd";
  VAE2_REQUIRE(x && ws && out && act_ok(xd), fn, "bad arguments");
  const int64_t total = act_elems(xd);
  const unsigned nb = reduce_blocks(total);
  hipStream_t s = as_stream(stream);
  VAE2_LAUNCH(sqdiff_partials_kernel, dim3(nb), dim3(256), 0, s, x, to_act(xd), target,
                     ws, FastDiv((uint32_t)xd->c));
  int rc = check_launch(fn);
  if (rc) return rc;
  VAE2_LAUNCH(finish_sum_kernel, dim3(1), dim3(256), 0, s, (const float*)ws, (int)nb,
                     scale, out, 0);
  return check_launch(fn);
}

int vae2_lsgan_bwd(const float* x, const vae2_act* xd, float target, const float* gout,
                   float scale, float* dx, const vae2_act* dxd, float beta, void* stream) {
  const char* fn = "vae2_lsgan_bwd";
  VAE2_REQUIRE(x && gout && dx && act_ok(xd) && act_ok(dxd), fn, "bad arguments");
  VAE2_REQUIRE(dxd->n == xd->n && dxd->h == xd->h && dxd->w == xd->w && dxd->c == xd->c, fn,
               "dx shape mismatch");
  const int64_t total = act_elems(xd);
  VAE2_LAUNCH(sqdiff_bwd_kernel, dim3(ew_blocks(total)), dim3(256), 0, as_stream(stream),
                     x, to_act(xd), target, gout, scale, dx, to_act(dxd), beta,
                     FastDiv((uint32_t)xd->c));
  return check_launch(fn);
}

int vae2_reparam_kl_fwd(const float* muvar, const vae2_act* md,
                        const float* eps, const vae2_act* ed, float* z,
                        const vae2_act* zd, int prior, float scale,
                        float* kl_out, int accumulate, float* ws, void* stream) {
  const char* fn = "vae2_reparam_kl_fwd";
  VAE2_REQUIRE(muvar && eps && z && kl_out && ws && act_ok(md) && act_ok(ed) && act_ok(zd), fn,
               "bad arguments");
  VAE2_REQUIRE(md->c == 2 * zd->c && ed->c == zd->c, fn, "channel mismatch");
  int64_t total = act_elems(zd);
  unsigned nb = reduce_blocks(total);
  hipStream_t s = as_stream(stream);
  VAE2_LAUNCH(reparam_kl_kernel, dim3(nb), dim3(256), 0, s, muvar, to_act(md), eps,
                     to_act(ed), z, to_act(zd), prior, ws, FastDiv((uint32_t)zd->c));
  int rc = check_launch(fn);
  if (rc) return rc;
  VAE2_LAUNCH(finish_sum_kernel, dim3(1), dim3(256), 0, s, (const float*)ws, (int)nb,
                     scale, kl_out, accumulate);
  return check_launch(fn);
}

int vae2_reparam_kl_bwd(const float* muvar, const vae2_act* md,
                        const float* eps, const vae2_act* ed, const float* dz,
                        const vae2_act* dzd, const float* gkl, float scale,
                        float* dmuvar, const vae2_act* dmd, void* stream) {
  const char* fn = "vae2_reparam_kl_bwd";
  VAE2_REQUIRE(muvar && eps && dmuvar && act_ok(md) && act_ok(ed) && act_ok(dmd), fn,
               "bad arguments");
  VAE2_REQUIRE(!dz || act_ok(dzd), fn, "bad dz descriptor");
  int64_t total = act_elems(ed);
  Act dza = dz ? to_act(dzd) : to_act(ed);
  VAE2_LAUNCH(reparam_kl_bwd_kernel, dim3(ew_blocks(total)), dim3(256), 0,
                     as_stream(stream), muvar, to_act(md), eps, to_act(ed), dz, dza, gkl, scale,
                     dmuvar, to_act(dmd), FastDiv((uint32_t)ed->c));
  return check_launch(fn);
}

int vae2_weighted_sum(int n, const float* const* terms, const float* lambdas,
                      float* total, void* stream) {
  const char* fn = "vae2_weighted_sum";
  VAE2_REQUIRE(n >= 1 && n <= 8 && terms && lambdas && total, fn, "bad arguments");
  WSum w{};
  w.n = n;
  for (int i = 0; i < n; ++i) {
    VAE2_REQUIRE(terms[i], fn, "null term");
    w.t[i] = terms[i];
    w.l[i] = lambdas[i];
  }
  VAE2_LAUNCH(weighted_sum_kernel, dim3(1), dim3(64), 0, as_stream(stream), w, total);
  return check_launch(fn);
}

int vae2_nonfinite_check(const float* x, int64_t n, int32_t* flag,
                         void* stream) {
  const char* fn = "vae2_nonfinite_check";
  VAE2_REQUIRE(x && flag && n >= 0, fn, "bad arguments");
  if (n == 0) return 0;
  VAE2_LAUNCH(nonfinite_kernel, dim3(ew_blocks(n, 256, 1024)), dim3(256), 0,
                     as_stream(stream), x, n, flag);
  return check_launch(fn);
}

int vae2_adam_step(float* p, const float* g, float* m, float* v, int64_t n,
                   float lr, float beta1, float beta2, float eps,
                   float weight_decay, int64_t step, void* stream) {
  const char* fn = "vae2_adam_step";
  VAE2_REQUIRE(p && g && m && v && n >= 0 && step >= 1, fn, "bad arguments");
  if (n == 0) return 0;
  double bc1 = 1.0 - pow((double)beta1, (double)step);
  double bc2 = 1.0 - pow((double)beta2, (double)step);
  float lr_corr = (float)((double)lr / bc1);
  float bc2s = (float)sqrt(bc2);
  VAE2_LAUNCH(adam_kernel, dim3(ew_blocks(n, 256, 4096)), dim3(256), 0,
                     as_stream(stream), p, g, m, v, n, lr_corr, beta1, beta2, eps,
                     weight_decay, bc2s);
  return check_launch(fn);
}

int vae2_adam_coeffs(double* state, float beta1, float beta2, float* coeffs,
                     void* stream) {
  const char* fn = "vae2_adam_coeffs";
  VAE2_REQUIRE(state && coeffs, fn, "null pointer");
  VAE2_LAUNCH(adam_coeffs_kernel, dim3(1), dim3(1), 0, as_stream(stream), state, beta1,
                     beta2, coeffs);
  return check_launch(fn);
}

int vae2_adam_step_dev(float* p, const float* g, float* m, float* v, int64_t n,
                       const float* coeffs, float beta1, float beta2, float eps,
                       float weight_decay, void* stream) {
  const char* fn = "vae2_adam_step_dev";
  VAE2_REQUIRE(p && g && m && v && coeffs && n >= 0, fn, "bad arguments");
  if (n == 0) return 0;
  VAE2_LAUNCH(adam_dev_kernel, dim3(ew_blocks(n, 256, 4096)), dim3(256), 0,
                     as_stream(stream), p, g, m, v, n, coeffs, beta1, beta2, eps, weight_decay);
  return check_launch(fn);
}

int vae2_scale(float* dst, const float* src, int64_t n, float scale,
               void* stream) {
  const char* fn = "vae2_scale";
  VAE2_REQUIRE(dst && src && n >= 0, fn, "bad arguments");
  if (n == 0) return 0;
  VAE2_LAUNCH(scale_kernel, dim3(ew_blocks(n, 256, 4096)), dim3(256), 0,
                     as_stream(stream), dst, src, n, scale);
  return check_launch(fn);
}

}  // extern "C"
