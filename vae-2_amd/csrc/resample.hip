// Bilinear resampling, multi-resolution fuse sums, code-map tiling, layout
// conversion and global average pooling for NHWC fp32 activations.
//
//   F.interpolate / F.upsample(mode='bilinear', align_corners=False)
//       enc_hrnet.py:242-245 (fuse), :835-837 / :893-895 / :951-953 (heads),
//       :1111-1113 (z-net)                              -> upsample fwd / bwd
//   HighResolutionModule fuse sum + ReLU :233-249      -> fuse_sum_relu
//   _gen_code_map + torch.cat :454-462, :819-827       -> codemap tile fwd / bwd
//   nn.AdaptiveAvgPool2d((1,1)) :1025                  -> global avgpool fwd / bwd
#include "common.h"

#include <cxxabi.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace vae2 {

// ------------------------------------------------------ launch log ----
static std::atomic<bool> g_klog{false};
static thread_local std::vector<const void*> g_klog_v;

void note_kernel(const void* host_fn) {
  if (g_klog.load(std::memory_order_relaxed)) g_klog_v.push_back(host_fn);
}

// "void vae2::dconv3_kernel<4, 2, false>(vae2::DConv)" -> "dconv3_kernel<4, 2, false>"
static std::string kernel_label(const void* fn) {
  const char* raw = hipKernelNameRefByPtr(fn, nullptr);
  if (!raw) return "?";
  int st = 0;
  char* dem = abi::__cxa_demangle(raw, nullptr, nullptr, &st);
  std::string s = (st == 0 && dem) ? dem : raw;
  std::free(dem);
  if (s.rfind("void ", 0) == 0) s = s.substr(5);
  int depth = 0;
  for (size_t i = 0; i < s.size(); ++i) {  // drop the parameter list
    if (s[i] == '<') ++depth;
    if (s[i] == '>') --depth;
    if (s[i] == '(' && depth == 0) { s = s.substr(0, i); break; }
  }
  size_t pos;
  while ((pos = s.find("vae2::")) != std::string::npos) s.erase(pos, 6);
  return s;
}

// ------------------------------------------------------------- errors ----
static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(const char* fn, const std::string& msg) {
  set_error(std::string(fn) + ": " + msg);
  return -22;
}

int check_launch(const char* fn) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(fn) + ": " + hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

// ------------------------------------------------- bilinear helpers ----
// (lerp_index: common.h)
__device__ __forceinline__ float bilinear_at(const float* __restrict__ x, const Act& xd,
                                             int64_t n, int oy, int ox, int c, float sh,
                                             float sw) {
  Lerp ly = lerp_index(oy, (int)xd.h, sh);
  Lerp lx = lerp_index(ox, (int)xd.w, sw);
  const float* base = x + n * xd.h * xd.w * xd.ps + c;
  float x00 = base[((int64_t)ly.i0 * xd.w + lx.i0) * xd.ps];
  float x01 = base[((int64_t)ly.i0 * xd.w + lx.i1) * xd.ps];
  float x10 = base[((int64_t)ly.i1 * xd.w + lx.i0) * xd.ps];
  float x11 = base[((int64_t)ly.i1 * xd.w + lx.i1) * xd.ps];
  return ly.l0 * (lx.l0 * x00 + lx.l1 * x01) + ly.l1 * (lx.l0 * x10 + lx.l1 * x11);
}

__global__ __launch_bounds__(256) void upsample_fwd_kernel(const float* __restrict__ x, Act xd,
                                                           float* __restrict__ y, Act yd,
                                                           float beta, FastDiv cdiv,
                                                           FastDiv wdiv, FastDiv hdiv) {
  const uint32_t C = (uint32_t)yd.c;
  const uint32_t total = (uint32_t)(yd.n * yd.h * yd.w) * C;
  const float sh = (float)xd.h / (float)yd.h;
  const float sw = (float)xd.w / (float)yd.w;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t p = cdiv.div(i);
    uint32_t c = i - p * C;
    uint32_t row = wdiv.div(p);
    uint32_t ox = p - row * (uint32_t)yd.w;
    uint32_t n = hdiv.div(row);
    uint32_t oy = row - n * (uint32_t)yd.h;
    float v = bilinear_at(x, xd, n, oy, ox, c, sh, sw);
    float* dst = y + (int64_t)p * yd.ps + c;
    *dst = (beta != 0.f) ? v + beta * *dst : v;
  }
}

// Adjoint: dx[n,iy,ix,c] = sum_{oy,ox} wy(oy,iy) wx(ox,ix) dy[n,oy,ox,c].
__global__ __launch_bounds__(256) void upsample_bwd_kernel(const float* __restrict__ dy, Act dyd,
                                                           float* __restrict__ dx, Act dxd,
                                                           float beta, FastDiv cdiv,
                                                           FastDiv wdiv, FastDiv hdiv) {
  const uint32_t C = (uint32_t)dxd.c;
  const uint32_t total = (uint32_t)(dxd.n * dxd.h * dxd.w) * C;
  const float sh = (float)dxd.h / (float)dyd.h;
  const float sw = (float)dxd.w / (float)dyd.w;
  const int OH = (int)dyd.h, OW = (int)dyd.w;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t p = cdiv.div(i);
    uint32_t c = i - p * C;
    uint32_t row = wdiv.div(p);
    int ix = (int)(p - row * (uint32_t)dxd.w);
    uint32_t n = hdiv.div(row);
    int iy = (int)(row - n * (uint32_t)dxd.h);
    // candidate output ranges (exactly re-checked by lerp_weight)
    int ylo = (int)floorf(((float)iy - 0.5f) / sh - 0.5f) - 1;
    int yhi = (int)ceilf(((float)iy + 1.5f) / sh - 0.5f) + 1;
    int xlo = (int)floorf(((float)ix - 0.5f) / sw - 0.5f) - 1;
    int xhi = (int)ceilf(((float)ix + 1.5f) / sw - 0.5f) + 1;
    if (ylo < 0) ylo = 0;
    if (xlo < 0) xlo = 0;
    if (yhi > OH - 1) yhi = OH - 1;
    if (xhi > OW - 1) xhi = OW - 1;
    // the last input row/col also collects every output beyond the range
    if (iy == (int)dxd.h - 1) yhi = OH - 1;
    if (ix == (int)dxd.w - 1) xhi = OW - 1;
    const float* base = dy + (int64_t)n * OH * OW * dyd.ps + c;
    float acc = 0.f;
    for (int oy = ylo; oy <= yhi; ++oy) {
      float wy = lerp_weight(oy, (int)dxd.h, sh, iy);
      if (wy == 0.f) continue;
      float accx = 0.f;
      for (int ox = xlo; ox <= xhi; ++ox) {
        float wx = lerp_weight(ox, (int)dxd.w, sw, ix);
        if (wx == 0.f) continue;
        accx += wx * base[((int64_t)oy * OW + ox) * dyd.ps];
      }
      acc += wy * accx;
    }
    float* dst = dx + (int64_t)p * dxd.ps + c;
    *dst = (beta != 0.f) ? acc + beta * *dst : acc;
  }
}

// The same adjoint, one thread per (input pixel, channel quad): 16-byte loads of dy
// (pixel strides are multiples of 4 floats) and the column weights of the window
// computed once per thread instead of once per (row, column).  Same summation order
// as upsample_bwd_kernel (row sums over ascending columns, then rows).  Windows wider
// than kUpW columns take the generic loop.
typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int kUpW = 24;

__global__ __launch_bounds__(256) void upsample_bwd4_kernel(const float* __restrict__ dy, Act dyd,
                                                            float* __restrict__ dx, Act dxd,
                                                            float beta, FastDiv qdiv,
                                                            FastDiv wdiv, FastDiv hdiv) {
  const uint32_t C = (uint32_t)dxd.c, Q = (C + 3) / 4;
  const uint32_t total = (uint32_t)(dxd.n * dxd.h * dxd.w) * Q;
  const float sh = (float)dxd.h / (float)dyd.h;
  const float sw = (float)dxd.w / (float)dyd.w;
  const int OH = (int)dyd.h, OW = (int)dyd.w;
  const int64_t ps = dyd.ps;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const uint32_t p = qdiv.div(i);
    const uint32_t c = 4 * (i - p * Q);
    const uint32_t row = wdiv.div(p);
    const int ix = (int)(p - row * (uint32_t)dxd.w);
    const uint32_t n = hdiv.div(row);
    const int iy = (int)(row - n * (uint32_t)dxd.h);
    int ylo = (int)floorf(((float)iy - 0.5f) / sh - 0.5f) - 1;
    int yhi = (int)ceilf(((float)iy + 1.5f) / sh - 0.5f) + 1;
    int xlo = (int)floorf(((float)ix - 0.5f) / sw - 0.5f) - 1;
    int xhi = (int)ceilf(((float)ix + 1.5f) / sw - 0.5f) + 1;
    if (ylo < 0) ylo = 0;
    if (xlo < 0) xlo = 0;
    if (yhi > OH - 1) yhi = OH - 1;
    if (xhi > OW - 1) xhi = OW - 1;
    if (iy == (int)dxd.h - 1) yhi = OH - 1;
    if (ix == (int)dxd.w - 1) xhi = OW - 1;
    const float* base = dy + (int64_t)n * OH * OW * ps + c;
    f4v acc = {0.f, 0.f, 0.f, 0.f};
    if (xhi - xlo < kUpW) {
      float wx[kUpW];
#pragma unroll
      for (int k = 0; k < kUpW; ++k)
        wx[k] = (xlo + k <= xhi) ? lerp_weight(xlo + k, (int)dxd.w, sw, ix) : 0.f;
      for (int oy = ylo; oy <= yhi; ++oy) {
        const float wy = lerp_weight(oy, (int)dxd.h, sh, iy);
        if (wy == 0.f) continue;
        const float* rp = base + ((int64_t)oy * OW + xlo) * ps;
        f4v ax = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < kUpW; ++k)
          if (wx[k] != 0.f) ax += wx[k] * *reinterpret_cast<const f4v*>(rp + k * ps);
        acc += wy * ax;
      }
    } else {
      for (int oy = ylo; oy <= yhi; ++oy) {
        const float wy = lerp_weight(oy, (int)dxd.h, sh, iy);
        if (wy == 0.f) continue;
        f4v ax = {0.f, 0.f, 0.f, 0.f};
        for (int ox = xlo; ox <= xhi; ++ox) {
          const float wxv = lerp_weight(ox, (int)dxd.w, sw, ix);
          if (wxv == 0.f) continue;
          ax += wxv * *reinterpret_cast<const f4v*>(base + ((int64_t)oy * OW + ox) * ps);
        }
        acc += wy * ax;
      }
    }
    float* dst = dx + (int64_t)p * dxd.ps + c;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c + k < C) dst[k] = (beta != 0.f) ? acc[k] + beta * dst[k] : acc[k];
  }
}

// The adjoint for up to 3 targets at exact 2, 4, 8 ratios (a fuse row's lower branches),
// one thread per (pixel, channel quad) so that narrow layers (18 channels) keep every
// lane busy: a horizontal pass of all targets (one launch) into a quad-padded workspace
// hb[s] = [n][H][zw][4Q], then a vertical pass of all targets (one launch), both with the
// static hat stencils.  dy is read once from HBM; hb (1/F of dy each) twice from L2.
struct UpAdjQ {
  const float* g;
  int64_t g_ps;
  int H, W, Q, C, nt;
  float* hb[3];
  float* dx[3];
  int64_t dx_ps[3];
  int zh[3], zw[3], lf[3];  // lf = log2 of the ratio (1..3)
  float beta[3];
  uint32_t cnt_h[3], cnt_v[3];
  FastDiv zwq[3], zh_d[3], q_d;
};

// sum_d hat_w(d, F) v[F*i + d] over a line of `len` points with stride `st`, edges folded.
// Every tap's load is unconditional (out-of-line taps read a clamped in-line point with
// weight 0): guarded loads were branched around one by one, each waited for in turn.
template <int F>
__device__ __forceinline__ f4v hat_adj(const float* line, int64_t st, int len, int i, int n_src) {
  constexpr int HF = F / 2;
  const int x0 = F * i;
  f4v v[4 * HF];
#pragma unroll
  for (int d = -HF; d < 3 * HF; ++d) {
    const int x = x0 + d;
    const int xc = x < 0 ? 0 : (x >= len ? len - 1 : x);
    v[d + HF] = *reinterpret_cast<const f4v*>(line + xc * st);
  }
  f4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int d = -HF; d < 3 * HF; ++d) {
    const int x = x0 + d;
    if (x >= 0 && x < len) acc += hat_w(d, F) * v[d + HF];
  }
  if (i == 0) {  // virtual source -1: points d - F
#pragma unroll
    for (int d = F; d < 3 * HF; ++d)
      acc += hat_w(d, F) * *reinterpret_cast<const f4v*>(line + (d - F) * st);
  }
  if (i == n_src - 1) {  // virtual source n_src: points len + d
#pragma unroll
    for (int d = -HF; d < 0; ++d)
      acc += hat_w(d, F) * *reinterpret_cast<const f4v*>(line + (len + d) * st);
  }
  return acc;
}

template <bool VERT>
__global__ __launch_bounds__(256) void up_adjq_kernel(UpAdjQ p) {
  const int s = blockIdx.y;
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= (VERT ? p.cnt_v[s] : p.cnt_h[s])) return;
  const int zw = p.zw[s], Q = p.Q, lf = p.lf[s];
  const uint32_t row = p.zwq[s].div(i);  // horizontal: n*H + oy; vertical: n*zh + iy
  const uint32_t r = i - row * (uint32_t)(zw * Q);
  const uint32_t ix = p.q_d.div(r);
  const uint32_t q = r - ix * (uint32_t)Q;
  const int64_t hrow = (int64_t)zw * 4 * Q;  // hb row stride
  if (!VERT) {
    const float* line = p.g + (int64_t)row * p.W * p.g_ps + 4 * q;
    const f4v acc = lf == 1   ? hat_adj<2>(line, p.g_ps, p.W, (int)ix, zw)
                    : lf == 2 ? hat_adj<4>(line, p.g_ps, p.W, (int)ix, zw)
                              : hat_adj<8>(line, p.g_ps, p.W, (int)ix, zw);
    *reinterpret_cast<f4v*>(p.hb[s] + (int64_t)row * hrow + 4 * (ix * Q + q)) = acc;
    return;
  }
  const uint32_t n = p.zh_d[s].div(row);
  const int iy = (int)(row - n * (uint32_t)p.zh[s]);
  const float* line = p.hb[s] + (int64_t)n * p.H * hrow + 4 * (ix * Q + q);
  const f4v acc = lf == 1   ? hat_adj<2>(line, hrow, p.H, iy, p.zh[s])
                  : lf == 2 ? hat_adj<4>(line, hrow, p.H, iy, p.zh[s])
                            : hat_adj<8>(line, hrow, p.H, iy, p.zh[s]);
  float* dst = p.dx[s] + ((int64_t)row * zw + ix) * p.dx_ps[s] + 4 * q;
  const float beta = p.beta[s];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if ((int)(4 * q) + k < p.C) dst[k] = (beta != 0.f) ? acc[k] + beta * dst[k] : acc[k];
}

struct FuseTerms {
  const float* x[4];
  Act d[4];
  const float* sv[4];  // BatchNorm (mean, invstd, scale, shift) applied to the term, or null
  int n;
};

// A term that is the pre-BN output r of a BatchNorm layer whose normalised output is never
// stored (a fuse unit's conv + BN, enc_hrnet.py:199-218): its values are fma(r, scale,
// shift) -- bn_apply's arithmetic, so the sum is the stored path's bit for bit.
__device__ __forceinline__ float term_at(const float* x, const float* sv, int64_t i, int c,
                                         int C) {
  const float v = x[i];
  return sv ? __builtin_fmaf(v, sv[2 * C + c], sv[3 * C + c]) : v;
}

__global__ __launch_bounds__(256) void fuse_sum_relu_kernel(FuseTerms t, float* __restrict__ y,
                                                            Act yd, FastDiv cdiv, FastDiv wdiv,
                                                            FastDiv hdiv) {
  const uint32_t C = (uint32_t)yd.c;
  const uint32_t total = (uint32_t)(yd.n * yd.h * yd.w) * C;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t p = cdiv.div(i);
    uint32_t c = i - p * C;
    uint32_t row = wdiv.div(p);
    uint32_t ox = p - row * (uint32_t)yd.w;
    uint32_t n = hdiv.div(row);
    uint32_t oy = row - n * (uint32_t)yd.h;
    // every term's loads first (a term's loads consumed inside its own branch were waited
    // for before the next term's went out: one round trip per term), then the arithmetic
    // in the same order as before (bit for bit)
    float xv[4][4], wt[4][4], scl[4], shf[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= t.n) break;
      const Act& d = t.d[k];
      const float* sv = t.sv[k];
      if (d.h == yd.h && d.w == yd.w) {
        xv[k][0] = t.x[k][(int64_t)p * d.ps + c];
      } else {
        const Lerp ly = lerp_index(oy, (int)d.h, (float)d.h / (float)yd.h);
        const Lerp lx = lerp_index(ox, (int)d.w, (float)d.w / (float)yd.w);
        const float* base = t.x[k] + (int64_t)n * d.h * d.w * d.ps + c;
        xv[k][0] = base[((int64_t)ly.i0 * d.w + lx.i0) * d.ps];
        xv[k][1] = base[((int64_t)ly.i0 * d.w + lx.i1) * d.ps];
        xv[k][2] = base[((int64_t)ly.i1 * d.w + lx.i0) * d.ps];
        xv[k][3] = base[((int64_t)ly.i1 * d.w + lx.i1) * d.ps];
        wt[k][0] = ly.l0; wt[k][1] = ly.l1; wt[k][2] = lx.l0; wt[k][3] = lx.l1;
      }
      if (sv) {
        scl[k] = sv[2 * C + c];
        shf[k] = sv[3 * C + c];
      }
    }
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= t.n) break;
      const Act& d = t.d[k];
      const bool bn = t.sv[k] != nullptr;
      float v;
      if (d.h == yd.h && d.w == yd.w) {
        v = bn ? __builtin_fmaf(xv[k][0], scl[k], shf[k]) : xv[k][0];
      } else {
        float q[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) q[e] = bn ? __builtin_fmaf(xv[k][e], scl[k], shf[k]) : xv[k][e];
        v = wt[k][0] * (wt[k][2] * q[0] + wt[k][3] * q[1]) +
            wt[k][1] * (wt[k][2] * q[2] + wt[k][3] * q[3]);
      }
      acc = (k == 0) ? v : acc + v;
    }
    y[(int64_t)p * yd.ps + c] = acc < 0.f ? 0.f : acc;  // NaN propagates (torch.relu)
  }
}

int g_fuse_quad = 1;  // vae2_conv2d_set_tune key 21: the quad form of the fuse sum (0: per channel)

// The same sum, a channel quad per thread (every term and y 16-byte aligned with pixel
// strides % 4 == 0): the pixel decode and the bilinear indices / weights are computed once
// per quad instead of once per channel, 16-byte loads through buffer resources (a partial
// quad reads its pixel's padding channels, whose sums are never stored), the stores of a
// partial quad limited to its valid channels (y may be a channel slice of a wider buffer).
// Per channel the arithmetic is fuse_sum_relu_kernel's, in the same order.
__global__ __launch_bounds__(256, 3) void fuse_sum_relu_q_kernel(FuseTerms t, float* __restrict__ y,
                                                              Act yd, FastDiv qdiv, FastDiv wdiv,
                                                              FastDiv hdiv) {
  const int C = (int)yd.c, c4 = (C + 3) >> 2;
  const uint32_t P = (uint32_t)(yd.n * yd.h * yd.w);
  const uint32_t total = P * (uint32_t)c4;
  __amdgpu_buffer_rsrc_t xr[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    xr[k] = make_rsrc(k < t.n ? t.x[k] : nullptr,
                      k < t.n ? (uint32_t)(t.d[k].n * t.d[k].h * t.d[k].w * t.d[k].ps * 4) : 0u);
  const __amdgpu_buffer_rsrc_t yr = make_rsrc(y, P * (uint32_t)yd.ps * 4u);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const uint32_t p = qdiv.div(i);
    const int c = 4 * (int)(i - p * (uint32_t)c4);
    const uint32_t row = wdiv.div(p);
    const uint32_t ox = p - row * (uint32_t)yd.w;
    const uint32_t n = hdiv.div(row);
    const uint32_t oy = row - n * (uint32_t)yd.h;
    // every term's loads first, then the arithmetic (fuse_sum_relu_kernel's order)
    f4 xv[4][4], scl[4], shf[4];
    float wt[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= t.n) break;
      const Act& d = t.d[k];
      const uint32_t ps4 = (uint32_t)d.ps * 4u, cb = (uint32_t)c * 4u;
      if (d.h == yd.h && d.w == yd.w) {
        xv[k][0] = load4(xr[k], p * ps4 + cb);
      } else {
        const Lerp ly = lerp_index((int)oy, (int)d.h, (float)d.h / (float)yd.h);
        const Lerp lx = lerp_index((int)ox, (int)d.w, (float)d.w / (float)yd.w);
        const uint32_t base = n * (uint32_t)(d.h * d.w);
        xv[k][0] = load4(xr[k], (base + (uint32_t)(ly.i0 * d.w + lx.i0)) * ps4 + cb);
        xv[k][1] = load4(xr[k], (base + (uint32_t)(ly.i0 * d.w + lx.i1)) * ps4 + cb);
        xv[k][2] = load4(xr[k], (base + (uint32_t)(ly.i1 * d.w + lx.i0)) * ps4 + cb);
        xv[k][3] = load4(xr[k], (base + (uint32_t)(ly.i1 * d.w + lx.i1)) * ps4 + cb);
        wt[k][0] = ly.l0; wt[k][1] = ly.l1; wt[k][2] = lx.l0; wt[k][3] = lx.l1;
      }
      if (const float* sv = t.sv[k]) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int ch = c + e < C ? c + e : C - 1;  // (clamped: the padding lanes are dropped)
          scl[k][e] = sv[2 * C + ch];
          shf[k][e] = sv[3 * C + ch];
        }
      }
    }
    f4 acc;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (k >= t.n) break;
        const Act& d = t.d[k];
        const bool bn = t.sv[k] != nullptr;
        float v;
        if (d.h == yd.h && d.w == yd.w) {
          v = bn ? __builtin_fmaf(xv[k][0][e], scl[k][e], shf[k][e]) : xv[k][0][e];
        } else {
          float q[4];
#pragma unroll
          for (int u = 0; u < 4; ++u)
            q[u] = bn ? __builtin_fmaf(xv[k][u][e], scl[k][e], shf[k][e]) : xv[k][u][e];
          v = wt[k][0] * (wt[k][2] * q[0] + wt[k][3] * q[1]) +
              wt[k][1] * (wt[k][2] * q[2] + wt[k][3] * q[3]);
        }
        a = (k == 0) ? v : a + v;
      }
      acc[e] = a < 0.f ? 0.f : a;  // NaN propagates (torch.relu)
    }
    store_quad(yr, (p * (uint32_t)yd.ps + (uint32_t)c) * 4u, acc, C - c < 4 ? C - c : 4);
  }
}

__global__ __launch_bounds__(256) void relu_bwd_kernel(const float* __restrict__ dy, Act dyd,
                                                       const float* __restrict__ y, Act yd,
                                                       float* __restrict__ g, Act gd,
                                                       FastDiv cdiv) {
  const uint32_t C = (uint32_t)yd.c;
  const uint32_t total = (uint32_t)(yd.n * yd.h * yd.w) * C;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t p = cdiv.div(i);
    uint32_t c = i - p * C;
    float v = dy[(int64_t)p * dyd.ps + c];
    g[(int64_t)p * gd.ps + c] = (y[(int64_t)p * yd.ps + c] > 0.f) ? v : 0.f;
  }
}

// g = dy * [y > 0] and g2 = g + beta2 * g2 (the same gradient handed to a second,
// accumulating consumer: ops.GradLink of a fuse input, no extra add kernel).
__global__ __launch_bounds__(256) void relu_bwd_dual_kernel(
    const float* __restrict__ dy, Act dyd, const float* __restrict__ y, Act yd,
    float* __restrict__ g, Act gd, float* __restrict__ g2, Act g2d, float beta2, FastDiv cdiv) {
  const uint32_t C = (uint32_t)yd.c;
  const uint32_t total = (uint32_t)(yd.n * yd.h * yd.w) * C;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t p = cdiv.div(i);
    uint32_t c = i - p * C;
    float v = dy[(int64_t)p * dyd.ps + c];
    v = (y[(int64_t)p * yd.ps + c] > 0.f) ? v : 0.f;
    g[(int64_t)p * gd.ps + c] = v;
    float* d2 = g2 + (int64_t)p * g2d.ps + c;
    *d2 = beta2 != 0.f ? v + beta2 * *d2 : v;
  }
}

// Channel-quad form (16-byte pixel rows): thread = (pixel, quad), one 16-byte load per
// operand and 16-byte stores (channels past C in the last quad untouched).
__global__ __launch_bounds__(256) void relu_bwd_dual_q_kernel(
    const float* __restrict__ dy, Act dyd, const float* __restrict__ y, Act yd,
    float* __restrict__ g, Act gd, float* __restrict__ g2, Act g2d, float beta2, FastDiv qdiv) {
  const int C = (int)yd.c, Q = (C + 3) >> 2;
  const uint32_t total = (uint32_t)(yd.n * yd.h * yd.w) * (uint32_t)Q;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const uint32_t p = qdiv.div(i);
    const int c = 4 * (int)(i - p * (uint32_t)Q);
    const f4 dv = *reinterpret_cast<const f4*>(dy + (int64_t)p * dyd.ps + c);
    const f4 yv = *reinterpret_cast<const f4*>(y + (int64_t)p * yd.ps + c);
    float* d2 = g2 + (int64_t)p * g2d.ps + c;
    f4 o2 = {0.f, 0.f, 0.f, 0.f};
    if (beta2 != 0.f) o2 = *reinterpret_cast<const f4*>(d2);
    f4 v;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = yv[k] > 0.f ? dv[k] : 0.f;
    float* d1 = g + (int64_t)p * gd.ps + c;
    if (c + 4 <= C) {
      *reinterpret_cast<f4*>(d1) = v;
      *reinterpret_cast<f4*>(d2) = beta2 != 0.f ? v + beta2 * o2 : v;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (c + k < C) {
          d1[k] = v[k];
          d2[k] = beta2 != 0.f ? v[k] + beta2 * o2[k] : v[k];
        }
    }
  }
}

__global__ __launch_bounds__(256) void copy_act_kernel(const float* __restrict__ x, Act xd,
                                                       float* __restrict__ y, Act yd, float beta,
                                                       FastDiv cdiv) {
  const uint32_t C = (uint32_t)xd.c;
  const uint32_t total = (uint32_t)(xd.n * xd.h * xd.w) * C;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t p = cdiv.div(i);
    uint32_t c = i - p * C;
    float v = x[(int64_t)p * xd.ps + c];
    float* dst = y + (int64_t)p * yd.ps + c;
    *dst = (beta != 0.f) ? v + beta * *dst : v;
  }
}

// y[n,h,w,c] = scale * v[n*vs + c] + beta * y
// y[n, iy, ix, c] (+)= scale * v[n][c] (* wr[iy] * wc[ix] when wr != null: the adjoint of
// a separably weighted spatial sum)
__global__ __launch_bounds__(256) void tile_kernel(const float* __restrict__ v, int64_t vs,
                                                   float* __restrict__ y, Act yd, float scale,
                                                   float beta, FastDiv cdiv, FastDiv hwdiv,
                                                   const float* __restrict__ wr = nullptr,
                                                   const float* __restrict__ wc = nullptr,
                                                   FastDiv wdiv = FastDiv()) {
  const uint32_t C = (uint32_t)yd.c;
  const uint32_t total = (uint32_t)(yd.n * yd.h * yd.w) * C;
  const uint32_t HW = (uint32_t)(yd.h * yd.w);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t p = cdiv.div(i);
    uint32_t c = i - p * C;
    uint32_t n = hwdiv.div(p);
    float val = scale * v[(int64_t)n * vs + c];
    if (wr) {
      const uint32_t q = p - n * HW, iy = wdiv.div(q);
      val *= wr[iy] * wc[q - iy * (uint32_t)yd.w];
    }
    float* dst = y + (int64_t)p * yd.ps + c;
    *dst = (beta != 0.f) ? val + beta * *dst : val;
  }
}

// Spatial sums per (n, c): stage 1 partials over pixel chunks.
__global__ __launch_bounds__(256) void spatial_partials_kernel(const float* __restrict__ x,
                                                               Act xd, int64_t ppb,
                                                               float* __restrict__ part,
                                                               const float* __restrict__ wr = nullptr,
                                                               const float* __restrict__ wc = nullptr) {
  __shared__ float red[256];
  const int C = (int)xd.c;
  const int64_t HW = xd.h * xd.w;
  const int64_t n = blockIdx.y;
  const int64_t p0 = blockIdx.x * ppb;
  int64_t p1 = p0 + ppb;
  if (p1 > HW) p1 = HW;
  const float* base = x + n * HW * xd.ps;
  float* out = part + (n * gridDim.x + blockIdx.x) * (int64_t)C;
  const int tid = threadIdx.x;
  if (C <= 256) {
    const int R = 256 / C, S = R * C;
    float s = 0.f;
    if (tid < S) {
      const int c = tid % C, rr = tid / C;
      if (wr) {  // (row, column) of p tracked incrementally: no 64-bit division per pixel
        const int W = (int)xd.w;
        int iy = (int)((p0 + rr) / W), ix = (int)((p0 + rr) - (int64_t)iy * W);
        for (int64_t p = p0 + rr; p < p1; p += R) {
          s += base[p * xd.ps + c] * (wr[iy] * wc[ix]);
          ix += R;
          while (ix >= W) {
            ix -= W;
            ++iy;
          }
        }
      } else {
        for (int64_t p = p0 + rr; p < p1; p += R) s += base[p * xd.ps + c];
      }
    }
    red[tid] = s;
    __syncthreads();
    if (tid < C) {
      float a = 0.f;
      for (int i = 0; i < R; ++i) a += red[tid + i * C];
      out[tid] = a;
    }
  } else {
    const int W = (int)xd.w;
    for (int c = tid; c < C; c += 256) {
      float s = 0.f;
      int iy = (int)(p0 / W), ix = (int)(p0 - (int64_t)iy * W);
      for (int64_t p = p0; p < p1; ++p) {
        s += base[p * xd.ps + c] * (wr ? wr[iy] * wc[ix] : 1.f);
        if (++ix == W) {
          ix = 0;
          ++iy;
        }
      }
      out[c] = s;
    }
  }
}

// stage 2: out[n*os + c] (+)= scale * sum_chunks part[n][chunk][c]
__global__ void spatial_finish_kernel(const float* __restrict__ part, int64_t chunks, int64_t N,
                                      int64_t C, float* out, int64_t os, float scale,
                                      int accumulate) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= N * C) return;
  int64_t n = i / C, c = i - n * C;
  float s = 0.f;
  for (int64_t k = 0; k < chunks; ++k) s += part[(n * chunks + k) * C + c];
  s *= scale;
  float* dst = out + n * os + c;
  *dst = accumulate ? *dst + s : s;
}

static int64_t spatial_chunks(const vae2_act* xd, int64_t* ppb_out) {
  int64_t HW = xd->h * xd->w;
  int64_t chunks = ceil_div(HW, 128);  // (512 / 64: 512 workgroups at 128x256 x 8 looped
  if (chunks > 256) chunks = 256;      //  16 dependent loads per thread, 56 us per call)
  int64_t ppb = ceil_div(HW, chunks);
  if (ppb_out) *ppb_out = ppb;
  return ceil_div(HW, ppb);
}

static int spatial_sum(const float* x, const vae2_act* xd, float* out, int64_t os,
                       float scale, int accumulate, float* part, int64_t ws_size,
                       hipStream_t s, const char* fn, const float* wr = nullptr,
                       const float* wc = nullptr) {
  int64_t ppb = 0;
  int64_t chunks = spatial_chunks(xd, &ppb);
  VAE2_REQUIRE(part && ws_size >= xd->n * chunks * xd->c, fn, "workspace too small");
  VAE2_LAUNCH(spatial_partials_kernel, dim3((unsigned)chunks, (unsigned)xd->n),
                     dim3(256), 0, s, x, to_act(xd), ppb, part, wr, wc);
  int rc = check_launch(fn);
  if (rc) return rc;
  int64_t nc = xd->n * xd->c;
  VAE2_LAUNCH(spatial_finish_kernel, dim3((unsigned)ceil_div(nc, 256)), dim3(256), 0, s,
                     (const float*)part, chunks, xd->n, xd->c, out, os, scale, accumulate);
  return check_launch(fn);
}

__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const float* __restrict__ x,
                                                           float* __restrict__ y, Act yd,
                                                           float beta, FastDiv cdiv,
                                                           FastDiv hwdiv) {
  const uint32_t C = (uint32_t)yd.c;
  const uint32_t HW = (uint32_t)(yd.h * yd.w);
  const uint32_t total = (uint32_t)yd.n * HW * C;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    // i indexes the NCHW source linearly: coalesced reads
    uint32_t nc = hwdiv.div(i);
    uint32_t hw = i - nc * HW;
    uint32_t n = cdiv.div(nc);
    uint32_t c = nc - n * C;
    float* dst = y + ((int64_t)n * HW + hw) * yd.ps + c;
    float v = x[i];
    *dst = (beta != 0.f) ? v + beta * *dst : v;
  }
}

__global__ __launch_bounds__(256) void nhwc_to_nchw_kernel(const float* __restrict__ x, Act xd,
                                                           float* __restrict__ y, float beta,
                                                           FastDiv cdiv, FastDiv hwdiv) {
  const uint32_t C = (uint32_t)xd.c;
  const uint32_t HW = (uint32_t)(xd.h * xd.w);
  const uint32_t total = (uint32_t)xd.n * HW * C;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    uint32_t nc = hwdiv.div(i);
    uint32_t hw = i - nc * HW;
    uint32_t n = cdiv.div(nc);
    uint32_t c = nc - n * C;
    float v = x[((int64_t)n * HW + hw) * xd.ps + c];
    y[i] = (beta != 0.f) ? v + beta * y[i] : v;
  }
}

static bool same_hw(const vae2_act* a, const vae2_act* b) {
  return a->n == b->n && a->h == b->h && a->w == b->w;
}

}  // namespace vae2

using namespace vae2;

extern "C" {

int vae2_abi_version(void) { return VAE2_ABI_VERSION; }

const char* vae2_last_error(void) { return g_last_error.c_str(); }

int vae2_kernel_log(int enable) {
  g_klog.store(enable != 0);
  g_klog_v.clear();
  return 0;
}

int64_t vae2_kernel_log_read(char* buf, int64_t len) {
  std::string out;
  for (size_t i = 0; i < g_klog_v.size(); ++i) {
    if (i) out += ';';
    out += kernel_label(g_klog_v[i]);
  }
  const int64_t n = (int64_t)g_klog_v.size();
  g_klog_v.clear();
  if (buf && len > 0) {
    const size_t m = out.size() < (size_t)(len - 1) ? out.size() : (size_t)(len - 1);
    std::memcpy(buf, out.data(), m);
    buf[m] = 0;
  }
  return n;
}

int vae2_upsample_bilinear_fwd(const float* x, const vae2_act* xd, float* y,
                               const vae2_act* yd, float beta, void* stream) {
  const char* fn = "vae2_upsample_bilinear_fwd";
  VAE2_REQUIRE(x && y && act_ok(xd) && act_ok(yd), fn, "bad arguments");
  VAE2_REQUIRE(xd->n == yd->n && xd->c == yd->c, fn, "n / c mismatch");
  int64_t total = act_elems(yd);
  VAE2_REQUIRE(total < (int64_t(1) << 31), fn, "tensor too large");
  VAE2_LAUNCH(upsample_fwd_kernel, dim3(ew_blocks(total)), dim3(256), 0,
                     as_stream(stream), x, to_act(xd), y, to_act(yd), beta,
                     FastDiv((uint32_t)yd->c), FastDiv((uint32_t)yd->w),
                     FastDiv((uint32_t)yd->h));
  return check_launch(fn);
}

int vae2_upsample_bilinear_bwd(const float* dy, const vae2_act* dyd, float* dx,
                               const vae2_act* dxd, float beta, void* stream) {
  const char* fn = "vae2_upsample_bilinear_bwd";
  VAE2_REQUIRE(dy && dx && act_ok(dyd) && act_ok(dxd), fn, "bad arguments");
  VAE2_REQUIRE(dxd->n == dyd->n && dxd->c == dyd->c, fn, "n / c mismatch");
  int64_t total = act_elems(dxd);
  VAE2_REQUIRE(total < (int64_t(1) << 31) && act_elems(dyd) < (int64_t(1) << 31), fn,
               "tensor too large");
  if (dyd->ps % 4 == 0 && (uintptr_t)dy % 16 == 0) {
    const int64_t quads = act_elems(dxd) / dxd->c * ((dxd->c + 3) / 4);
    VAE2_LAUNCH(upsample_bwd4_kernel, dim3(ew_blocks(quads)), dim3(256), 0,
                       as_stream(stream), dy, to_act(dyd), dx, to_act(dxd), beta,
                       FastDiv((uint32_t)((dxd->c + 3) / 4)), FastDiv((uint32_t)dxd->w),
                       FastDiv((uint32_t)dxd->h));
    return check_launch(fn);
  }
  VAE2_LAUNCH(upsample_bwd_kernel, dim3(ew_blocks(total)), dim3(256), 0,
                     as_stream(stream), dy, to_act(dyd), dx, to_act(dxd), beta,
                     FastDiv((uint32_t)dxd->c), FastDiv((uint32_t)dxd->w),
                     FastDiv((uint32_t)dxd->h));
  return check_launch(fn);
}

// log2 of an exact power-of-two ratio in {2, 4, 8}, else 0.
static int pow2_ratio(int64_t big, int64_t small) {
  for (int k = 1; k <= 3; ++k)
    if (big == small << k) return k;
  return 0;
}

int64_t vae2_upsample_bilinear_bwd_pow2_ws_size(const vae2_act* dyd, int n,
                                                const vae2_act* dxds) {
  if (!act_ok(dyd) || n < 1 || n > 3 || !dxds) return -1;
  const int64_t Q = (dyd->c + 3) / 4;
  int64_t t = 0;
  for (int s = 0; s < n; ++s) {
    const vae2_act* d = &dxds[s];
    const int k = pow2_ratio(dyd->w, d->w);
    if (!act_ok(d) || !k || pow2_ratio(dyd->h, d->h) != k || d->n != dyd->n || d->c != dyd->c)
      return -1;
    t += dyd->n * dyd->h * d->w * 4 * Q;
  }
  return t;
}

int vae2_upsample_bilinear_bwd_pow2(const float* dy, const vae2_act* dyd, int n,
                                    float* const* dxs, const vae2_act* dxds,
                                    const float* betas, float* ws, int64_t ws_size,
                                    void* stream) {
  const char* fn = "vae2_upsample_bilinear_bwd_pow2";
  VAE2_REQUIRE(dy && act_ok(dyd) && n >= 1 && n <= 3 && dxs && dxds && ws, fn,
               "bad arguments");
  const int64_t need = vae2_upsample_bilinear_bwd_pow2_ws_size(dyd, n, dxds);
  VAE2_REQUIRE(need >= 0, fn, "targets are not exact 2 / 4 / 8 downsamplings of dy");
  VAE2_REQUIRE(ws_size >= need, fn, "workspace too small");
  VAE2_REQUIRE(dyd->ps % 4 == 0 && (uintptr_t)dy % 16 == 0 && (uintptr_t)ws % 16 == 0, fn,
               "dy and ws must be 16-byte aligned with a pixel stride of 4k");
  hipStream_t st = as_stream(stream);
  // one launch, dy read once (heads.hip's band kernel) where the targets are 2 / 4 / 8 in
  // order and the rows are 64-pixel chunks
  if (adj3_fuse_launch(dy, dyd, n, dxs, dxds, betas, st) == 0) return check_launch(fn);
  UpAdjQ p{};
  p.g = dy; p.g_ps = dyd->ps; p.H = (int)dyd->h; p.W = (int)dyd->w; p.C = (int)dyd->c;
  p.Q = (p.C + 3) / 4; p.nt = n; p.q_d = FastDiv((uint32_t)p.Q);
  float* hb = ws;
  uint32_t mh = 0, mv = 0;
  for (int s = 0; s < n; ++s) {
    const vae2_act* d = &dxds[s];
    VAE2_REQUIRE(dxs[s], fn, "null target");
    const int64_t ch = dyd->n * dyd->h * d->w * p.Q, cv = dyd->n * d->h * d->w * p.Q;
    VAE2_REQUIRE(ch < (int64_t(1) << 31), fn, "tensor too large");
    p.dx[s] = dxs[s]; p.dx_ps[s] = d->ps; p.zh[s] = (int)d->h; p.zw[s] = (int)d->w;
    p.lf[s] = pow2_ratio(dyd->w, d->w);
    p.beta[s] = betas ? betas[s] : 0.f;
    p.cnt_h[s] = (uint32_t)ch; p.cnt_v[s] = (uint32_t)cv;
    p.zwq[s] = FastDiv((uint32_t)(d->w * p.Q)); p.zh_d[s] = FastDiv((uint32_t)d->h);
    p.hb[s] = hb;
    hb += dyd->n * dyd->h * d->w * 4 * p.Q;
    if (p.cnt_h[s] > mh) mh = p.cnt_h[s];
    if (p.cnt_v[s] > mv) mv = p.cnt_v[s];
  }
  VAE2_LAUNCH(up_adjq_kernel<false>, dim3((mh + 255) / 256, n), dim3(256), 0, st, p);
  int rc = check_launch(fn);
  if (rc) return rc;
  VAE2_LAUNCH(up_adjq_kernel<true>, dim3((mv + 255) / 256, n), dim3(256), 0, st, p);
  return check_launch(fn);
}

static int fuse_sum_relu_impl(int n, const float* const* xs, const vae2_act* xds,
                              const float* const* saves, float* y, const vae2_act* yd,
                              void* stream, const char* fn) {
  VAE2_REQUIRE(n >= 1 && n <= 4 && xs && xds && y && act_ok(yd), fn, "bad arguments");
  FuseTerms t{};
  t.n = n;
  for (int k = 0; k < n; ++k) {
    VAE2_REQUIRE(xs[k] && act_ok(&xds[k]), fn, "bad term");
    VAE2_REQUIRE(xds[k].n == yd->n && xds[k].c == yd->c, fn, "term n / c mismatch");
    VAE2_REQUIRE(xds[k].h <= yd->h && xds[k].w <= yd->w, fn, "terms cannot be downsampled");
    t.x[k] = xs[k];
    t.d[k] = to_act(&xds[k]);
    t.sv[k] = saves ? saves[k] : nullptr;
  }
  int64_t total = act_elems(yd);
  VAE2_REQUIRE(total < (int64_t(1) << 31), fn, "tensor too large");
  // the quad form: 16-byte aligned terms and output, pixel strides % 4 == 0, every extent
  // addressable with 32-bit buffer offsets
  bool quad = g_fuse_quad && (uintptr_t)y % 16 == 0 && yd->ps % 4 == 0 &&
              act_pixels(yd) * yd->ps * 4 < (int64_t(1) << 32);
  for (int k = 0; k < n && quad; ++k)
    quad = (uintptr_t)xs[k] % 16 == 0 && xds[k].ps % 4 == 0 &&
           act_pixels(&xds[k]) * xds[k].ps * 4 < (int64_t(1) << 32);
  if (quad) {
    const int64_t quads = act_pixels(yd) * ((yd->c + 3) / 4);
    VAE2_LAUNCH(fuse_sum_relu_q_kernel, dim3(ew_blocks(quads, 256, 8192)), dim3(256), 0,
                as_stream(stream), t, y, to_act(yd), FastDiv((uint32_t)((yd->c + 3) / 4)),
                FastDiv((uint32_t)yd->w), FastDiv((uint32_t)yd->h));
    return check_launch(fn);
  }
  // (grid-striding over 8192 blocks: one element per thread measured 27 -> 33 us per
  // launch in the step trace -- the per-thread index setup is amortised over 2-3 elements)
  VAE2_LAUNCH(fuse_sum_relu_kernel, dim3(ew_blocks(total, 256, 8192)), dim3(256), 0,
                     as_stream(stream), t, y, to_act(yd), FastDiv((uint32_t)yd->c),
                     FastDiv((uint32_t)yd->w), FastDiv((uint32_t)yd->h));
  return check_launch(fn);
}

int vae2_fuse_sum_relu(int n, const float* const* xs, const vae2_act* xds,
                       float* y, const vae2_act* yd, void* stream) {
  return fuse_sum_relu_impl(n, xs, xds, nullptr, y, yd, stream, "vae2_fuse_sum_relu");
}

int vae2_fuse_sum_relu_bn(int n, const float* const* xs, const vae2_act* xds,
                          const float* const* saves, float* y, const vae2_act* yd,
                          void* stream) {
  return fuse_sum_relu_impl(n, xs, xds, saves, y, yd, stream, "vae2_fuse_sum_relu_bn");
}

int vae2_relu_bwd(const float* dy, const vae2_act* dyd, const float* y,
                  const vae2_act* yd, float* g, const vae2_act* gd,
                  void* stream) {
  const char* fn = "vae2_relu_bwd";
  VAE2_REQUIRE(dy && y && g && act_ok(dyd) && act_ok(yd) && act_ok(gd), fn, "bad arguments");
  VAE2_REQUIRE(same_hw(dyd, yd) && same_hw(yd, gd) && dyd->c == yd->c && gd->c == yd->c, fn,
               "shape mismatch");
  int64_t total = act_elems(yd);
  VAE2_LAUNCH(relu_bwd_kernel, dim3(ew_blocks(total)), dim3(256), 0, as_stream(stream),
                     dy, to_act(dyd), y, to_act(yd), g, to_act(gd), FastDiv((uint32_t)yd->c));
  return check_launch(fn);
}

int vae2_relu_bwd_dual(const float* dy, const vae2_act* dyd, const float* y,
                       const vae2_act* yd, float* g, const vae2_act* gd, float* g2,
                       const vae2_act* g2d, float beta2, void* stream) {
  const char* fn = "vae2_relu_bwd_dual";
  VAE2_REQUIRE(dy && y && g && g2 && act_ok(dyd) && act_ok(yd) && act_ok(gd) && act_ok(g2d),
               fn, "bad arguments");
  VAE2_REQUIRE(same_hw(dyd, yd) && same_hw(yd, gd) && same_hw(yd, g2d) && dyd->c == yd->c &&
                   gd->c == yd->c && g2d->c == yd->c, fn, "shape mismatch");
  int64_t total = act_elems(yd);
  auto q16 = [](const float* ptr, const vae2_act* d) {
    return ((uintptr_t)ptr % 16 == 0) && d->ps % 4 == 0;
  };
  if (g_relu_dual_q && q16(dy, dyd) && q16(y, yd) && q16(g, gd) && q16(g2, g2d)) {
    const int64_t quads = act_pixels(yd) * ((yd->c + 3) / 4);
    VAE2_LAUNCH(relu_bwd_dual_q_kernel, dim3(ew_blocks(quads)), dim3(256), 0,
                as_stream(stream), dy, to_act(dyd), y, to_act(yd), g, to_act(gd), g2,
                to_act(g2d), beta2, FastDiv((uint32_t)((yd->c + 3) / 4)));
    return check_launch(fn);
  }
  VAE2_LAUNCH(relu_bwd_dual_kernel, dim3(ew_blocks(total)), dim3(256), 0, as_stream(stream),
              dy, to_act(dyd), y, to_act(yd), g, to_act(gd), g2, to_act(g2d), beta2,
              FastDiv((uint32_t)yd->c));
  return check_launch(fn);
}

int vae2_copy_act(const float* x, const vae2_act* xd, float* y,
                  const vae2_act* yd, float beta, void* stream) {
  const char* fn = "vae2_copy_act";
  VAE2_REQUIRE(x && y && act_ok(xd) && act_ok(yd), fn, "bad arguments");
  VAE2_REQUIRE(same_hw(xd, yd) && xd->c == yd->c, fn, "shape mismatch");
  int64_t total = act_elems(xd);
  VAE2_LAUNCH(copy_act_kernel, dim3(ew_blocks(total)), dim3(256), 0, as_stream(stream),
                     x, to_act(xd), y, to_act(yd), beta, FastDiv((uint32_t)xd->c));
  return check_launch(fn);
}

int vae2_codemap_tile_fwd(const float* v, int64_t vs, float* y,
                          const vae2_act* yd, void* stream) {
  const char* fn = "vae2_codemap_tile_fwd";
  VAE2_REQUIRE(v && y && act_ok(yd) && vs >= yd->c, fn, "bad arguments");
  int64_t total = act_elems(yd);
  VAE2_LAUNCH(tile_kernel, dim3(ew_blocks(total)), dim3(256), 0, as_stream(stream), v,
                     vs, y, to_act(yd), 1.f, 0.f, FastDiv((uint32_t)yd->c),
                     FastDiv((uint32_t)(yd->h * yd->w)));
  return check_launch(fn);
}

int64_t vae2_spatial_ws_size(const vae2_act* xd) {
  if (!act_ok(xd)) return 0;
  return xd->n * spatial_chunks(xd, nullptr) * xd->c;
}

int vae2_codemap_tile_bwd(const float* dy, const vae2_act* dyd, float* dv,
                          int64_t vs, int accumulate, float* ws, int64_t ws_size,
                          void* stream) {
  const char* fn = "vae2_codemap_tile_bwd";
  VAE2_REQUIRE(dy && dv && act_ok(dyd) && vs >= dyd->c, fn, "bad arguments");
  return spatial_sum(dy, dyd, dv, vs, 1.f, accumulate, ws, ws_size, as_stream(stream), fn);
}

int vae2_nchw_to_nhwc(const float* x, float* y, const vae2_act* yd,
                      float beta, void* stream) {
  const char* fn = "vae2_nchw_to_nhwc";
  VAE2_REQUIRE(x && y && act_ok(yd), fn, "bad arguments");
  int64_t total = act_elems(yd);
  VAE2_LAUNCH(nchw_to_nhwc_kernel, dim3(ew_blocks(total)), dim3(256), 0,
                     as_stream(stream), x, y, to_act(yd), beta, FastDiv((uint32_t)yd->c),
                     FastDiv((uint32_t)(yd->h * yd->w)));
  return check_launch(fn);
}

int vae2_nhwc_to_nchw(const float* x, const vae2_act* xd, float* y,
                      float beta, void* stream) {
  const char* fn = "vae2_nhwc_to_nchw";
  VAE2_REQUIRE(x && y && act_ok(xd), fn, "bad arguments");
  int64_t total = act_elems(xd);
  VAE2_LAUNCH(nhwc_to_nchw_kernel, dim3(ew_blocks(total)), dim3(256), 0,
                     as_stream(stream), x, to_act(xd), y, beta, FastDiv((uint32_t)xd->c),
                     FastDiv((uint32_t)(xd->h * xd->w)));
  return check_launch(fn);
}

int vae2_global_avgpool_fwd(const float* x, const vae2_act* xd, float* y,
                            const vae2_act* yd, float* ws, int64_t ws_size,
                            void* stream) {
  const char* fn = "vae2_global_avgpool_fwd";
  VAE2_REQUIRE(x && y && act_ok(xd) && act_ok(yd), fn, "bad arguments");
  VAE2_REQUIRE(yd->h == 1 && yd->w == 1 && yd->n == xd->n && yd->c == xd->c, fn,
               "output must be (n, 1, 1, c)");
  return spatial_sum(x, xd, y, yd->ps, 1.f / (float)(xd->h * xd->w), 0, ws, ws_size,
                     as_stream(stream), fn);
}

int vae2_weighted_avgpool_fwd(const float* x, const vae2_act* xd, const float* wr,
                              const float* wc, float scale, float* y, const vae2_act* yd,
                              float* ws, int64_t ws_size, void* stream) {
  const char* fn = "vae2_weighted_avgpool_fwd";
  VAE2_REQUIRE(x && y && wr && wc && act_ok(xd) && act_ok(yd), fn, "bad arguments");
  VAE2_REQUIRE(yd->h == 1 && yd->w == 1 && yd->n == xd->n && yd->c == xd->c, fn,
               "output must be (n, 1, 1, c)");
  return spatial_sum(x, xd, y, yd->ps, scale, 0, ws, ws_size, as_stream(stream), fn, wr, wc);
}

int vae2_weighted_avgpool_bwd(const float* dy, const vae2_act* dyd, const float* wr,
                              const float* wc, float scale, float* dx, const vae2_act* dxd,
                              float beta, void* stream) {
  const char* fn = "vae2_weighted_avgpool_bwd";
  VAE2_REQUIRE(dy && dx && wr && wc && act_ok(dyd) && act_ok(dxd), fn, "bad arguments");
  VAE2_REQUIRE(dyd->h == 1 && dyd->w == 1 && dyd->n == dxd->n && dyd->c == dxd->c, fn,
               "dy must be (n, 1, 1, c)");
  int64_t total = act_elems(dxd);
  VAE2_LAUNCH(tile_kernel, dim3(ew_blocks(total)), dim3(256), 0, as_stream(stream), dy,
              dyd->ps, dx, to_act(dxd), scale, beta, FastDiv((uint32_t)dxd->c),
              FastDiv((uint32_t)(dxd->h * dxd->w)), wr, wc, FastDiv((uint32_t)dxd->w));
  return check_launch(fn);
}

int vae2_global_avgpool_bwd(const float* dy, const vae2_act* dyd, float* dx,
                            const vae2_act* dxd, float beta, void* stream) {
  const char* fn = "vae2_global_avgpool_bwd";
  VAE2_REQUIRE(dy && dx && act_ok(dyd) && act_ok(dxd), fn, "bad arguments");
  VAE2_REQUIRE(dyd->h == 1 && dyd->w == 1 && dyd->n == dxd->n && dyd->c == dxd->c, fn,
               "dy must be (n, 1, 1, c)");
  int64_t total = act_elems(dxd);
  VAE2_LAUNCH(tile_kernel, dim3(ew_blocks(total)), dim3(256), 0, as_stream(stream), dy,
                     dyd->ps, dx, to_act(dxd), 1.f / (float)(dxd->h * dxd->w), beta,
                     FastDiv((uint32_t)dxd->c), FastDiv((uint32_t)(dxd->h * dxd->w)));
  return check_launch(fn);
}

}  // extern "C"
