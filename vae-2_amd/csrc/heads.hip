// Output stage of the HRNet heads: BatchNorm-apply + ReLU + the final narrow 1x1 conv
// (270 -> NUM_CLASSES), forward and backward, without materialising the ReLU output.
//
//   last_layer = Conv1x1(C->C, bias) -> BatchNorm2d -> ReLU -> Conv1x1(C->CO, bias)
//   (enc_hrnet.py:323-370 / :598-750; applied at :839-847, :897-905, :955-963)
//
// The wide 1x1 conv itself runs per branch (vae2_conv2d_fwd at the branch resolution,
// then upsum_kernel below: full-resolution block + upsampled branch terms + bias + BN
// statistics); the output-stage kernels take its pre-BN output y, the BN coefficients and
//   forward   out[p][o] = b2[o] + sum_c w2[o][c] * relu(y[p][c]*scale[c] + shift[c])
//   backward  g[p][c]  = (sum_o w2[o][c] * dout[p][o]) * [h > 0]      (h = ReLU input)
//             reduce:  sum_p g, sum_p g*xhat (BN backward sums), dW2, db2
//             apply:   dy = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat)), sum_p dy (conv bias)
// Each pass reads y once (16-byte NHWC quads); h and g are recomputed in registers.
// Reductions are two-level with fixed orders (deterministic).
#include "common.h"

namespace vae2 {


constexpr int kHeadMaxOut = 4;
constexpr int64_t kHeadMaxPpb = 2048;  // pixels per block of the backward passes (LDS dout)

// The block's dout rows [p0, p1) x CO, staged once in LDS (every channel quad of a pixel
// reads the same CO values: one coalesced pass instead of CO scalar loads per quad)
template <int CO>
__device__ __forceinline__ void head_stage_dout(float* sd, const float* dout, const Act& dod,
                                                int64_t p0, int64_t p1) {
  const int n = (int)(p1 - p0) * CO;
  for (int i = threadIdx.x; i < n; i += 256) {
    const int pp = i / CO, o = i - pp * CO;
    sd[i] = dout[(p0 + pp) * dod.ps + o];
  }
}

__device__ __forceinline__ f4 hld4(const float* p) { return *reinterpret_cast<const f4*>(p); }

// The wide conv's output y lives in a 64-channel-blocked layout ("B64"):
//   element (p, c) at y[(c / 64) * P * 64 + p * 64 + c % 64],  P = N*H*W pixels,
// so a workgroup producing a 64-channel block of a pixel run writes one contiguous
// region (NHWC rows of C = 270 would be written in partial 128-byte lines).
__device__ __forceinline__ const float* yb_at(const float* y, int64_t P, int64_t p, int c) {
  return y + (int64_t)(c >> 6) * P * 64 + p * 64 + (c & 63);
}

__device__ __forceinline__ f4 hchan4(const float* a, int c, int C) {
  f4 v;
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = (c + k < C) ? a[c + k] : 0.f;
  return v;
}

// Forward: 16 lanes per pixel (lane l takes channel quads l, l+16, ...), 16 pixels per
// block pass; the per-channel coefficients and W2 live in LDS as quads.
template <int CO>
__global__ __launch_bounds__(256) void head_out_fwd_kernel(
    const float* __restrict__ y, Act yd, const float* __restrict__ save,
    const float* __restrict__ w2, const float* __restrict__ b2, float* __restrict__ out,
    Act od) {
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  const int C = (int)yd.c, c4 = (C + 3) >> 2;
  f4* ssc = reinterpret_cast<f4*>(hsm);
  f4* ssh = ssc + c4;
  f4* sw = ssh + c4;  // [CO][c4]
  for (int q = threadIdx.x; q < c4; q += 256) {
    ssc[q] = hchan4(save + 2 * C, 4 * q, C);
    ssh[q] = hchan4(save + 3 * C, 4 * q, C);
#pragma unroll
    for (int o = 0; o < CO; ++o) sw[o * c4 + q] = hchan4(w2 + (int64_t)o * C, 4 * q, C);
  }
  __syncthreads();
  const int l = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int64_t P = yd.n * yd.h * yd.w;
  for (int64_t p = (int64_t)blockIdx.x * 16 + grp; p < P; p += (int64_t)gridDim.x * 16) {
    float acc[CO];
#pragma unroll
    for (int o = 0; o < CO; ++o) acc[o] = 0.f;
    // up to kHeadQU quads per lane with their loads in flight together (the same
    // quad order as one at a time)
    constexpr int kHeadQU = 5;
    for (int q0 = l; q0 < c4; q0 += 16 * kHeadQU) {
      f4 vv[kHeadQU];
#pragma unroll
      for (int u = 0; u < kHeadQU; ++u) {
        const int q = q0 + 16 * u;
        vv[u] = q < c4 ? hld4(yb_at(y, P, p, 4 * q)) : f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < kHeadQU; ++u) {
        const int q = q0 + 16 * u;
        if (q >= c4) break;
        const f4 v = vv[u];
        const f4 a = ssc[q], b = ssh[q];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float h = __builtin_fmaf(v[k], a[k], b[k]);
          h = (4 * q + k < C && !(h < 0.f)) ? h : 0.f;  // NaN propagates
#pragma unroll
          for (int o = 0; o < CO; ++o) acc[o] += h * sw[o * c4 + q][k];
        }
      }
    }
#pragma unroll
    for (int o = 0; o < CO; ++o) {
      acc[o] += __shfl_xor(acc[o], 8, 16);
      acc[o] += __shfl_xor(acc[o], 4, 16);
      acc[o] += __shfl_xor(acc[o], 2, 16);
      acc[o] += __shfl_xor(acc[o], 1, 16);
    }
    if (l == 0) {
#pragma unroll
      for (int o = 0; o < CO; ++o) out[p * od.ps + o] = acc[o] + (b2 ? b2[o] : 0.f);
    }
  }
}

// Per-thread state of the backward passes: thread (r, q) owns channels 4q..4q+3 and
// walks pixels p0 + r, p0 + r + rows, ... of its block's pixel range.
struct HeadCoef {
  f4 mean, invstd, sc, sh;
};

__device__ __forceinline__ HeadCoef head_coef(const float* save, int c, int C) {
  HeadCoef h;
  h.mean = hchan4(save, c, C);
  h.invstd = hchan4(save + C, c, C);
  h.sc = hchan4(save + 2 * C, c, C);
  h.sh = hchan4(save + 3 * C, c, C);
  return h;
}

// Partial-row columns: [0,C) sum g | [C,2C) sum g*xhat | [2C, 2C+CO*C) dW2[o][c] | CO x db2
template <int CO, int U = 2>
__global__ __launch_bounds__(256) void head_out_bwd_reduce_kernel(
    const float* __restrict__ y, Act yd, const float* __restrict__ save,
    const float* __restrict__ w2, const float* __restrict__ dout, Act dod, int64_t ppb,
    int rows, float* __restrict__ part) {
  extern __shared__ float red[];  // [rows][NC], then the dout rows [ppb][CO]
  const int C = (int)yd.c, c4 = (C + 3) >> 2;
  const int NC = 2 * C + CO * C + CO;
  const int tid = threadIdx.x;
  const int64_t P = yd.n * yd.h * yd.w;
  const int64_t p0 = blockIdx.x * ppb;
  const int64_t p1 = p0 + ppb < P ? p0 + ppb : P;
  const int r = tid / c4, q = tid - r * c4, c = 4 * q;
  float* sd = red + rows * NC;
  head_stage_dout<CO>(sd, dout, dod, p0, p1);
  __syncthreads();
  if (tid < rows * c4) {
    const HeadCoef hc = head_coef(save, c, C);
    f4 wv[CO];
#pragma unroll
    for (int o = 0; o < CO; ++o) wv[o] = hchan4(w2 + (int64_t)o * C, c, C);
    f4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
    f4 dw[CO];
    float db[CO];
#pragma unroll
    for (int o = 0; o < CO; ++o) { dw[o] = s0; db[o] = 0.f; }
    // U pixels in flight per thread (2: 4 waves/SIMD, 120 -> 95 us per head in round 2)
    for (int64_t pb = p0 + r; pb < p1; pb += U * rows) {
      f4 vv[U];
      float dd[U][CO];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t p = pb + u * rows;
        const bool ok = p < p1;
        vv[u] = ok ? hld4(yb_at(y, P, p, c)) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int o = 0; o < CO; ++o) dd[u][o] = ok ? sd[(p - p0) * CO + o] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const f4 v = vv[u];
        const float* d = dd[u];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float h = __builtin_fmaf(v[k], hc.sc[k], hc.sh[k]);
          const bool m = h > 0.f;
          h = m ? h : 0.f;
          float dh = 0.f;
#pragma unroll
          for (int o = 0; o < CO; ++o) dh += wv[o][k] * d[o];
          const float g = m ? dh : 0.f;
          s0[k] += g;
          s1[k] += g * (v[k] - hc.mean[k]) * hc.invstd[k];
#pragma unroll
          for (int o = 0; o < CO; ++o) dw[o][k] += d[o] * h;
        }
#pragma unroll
        for (int o = 0; o < CO; ++o) db[o] += d[o];
      }
    }
    float* rr = red + r * NC;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (c + k >= C) break;
      rr[c + k] = s0[k];
      rr[C + c + k] = s1[k];
#pragma unroll
      for (int o = 0; o < CO; ++o) rr[2 * C + o * C + c + k] = dw[o][k];
    }
    if (q == 0) {
#pragma unroll
      for (int o = 0; o < CO; ++o) rr[2 * C + CO * C + o] = db[o];
    }
  }
  __syncthreads();
  for (int col = tid; col < NC; col += 256) {
    float a = 0.f;
    for (int i = 0; i < rows; ++i) a += red[i * NC + col];
    part[(int64_t)blockIdx.x * NC + col] = a;
  }
}

// Column sums of the reduce partials (lane = column; 16 waves over rows with four
// independent accumulators each, in double; combined in a fixed order) routed to their
// destinations.
__global__ __launch_bounds__(1024) void head_bwd_colsum_kernel(
    const float* __restrict__ part, int nrows, int C, int CO, double* __restrict__ sums,
    float* dgamma, float* dbeta, float* dw2, float* db2) {
  __shared__ double red[16][64];
  const int NC = 2 * C + CO * C + CO;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (col < NC) {
    int i = wave;
    for (; i + 48 < nrows; i += 64) {
      s0 += (double)part[(int64_t)i * NC + col];
      s1 += (double)part[(int64_t)(i + 16) * NC + col];
      s2 += (double)part[(int64_t)(i + 32) * NC + col];
      s3 += (double)part[(int64_t)(i + 48) * NC + col];
    }
    for (; i < nrows; i += 16) s0 += (double)part[(int64_t)i * NC + col];
  }
  red[wave][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (wave != 0 || col >= NC) return;
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < 16; ++w) s += red[w][lane];
  if (col < C) {
    sums[col] = s;
    if (dbeta) dbeta[col] += (float)s;
  } else if (col < 2 * C) {
    sums[col] = s;
    if (dgamma) dgamma[col - C] += (float)s;
  } else if (col < 2 * C + CO * C) {
    if (dw2) dw2[col - 2 * C] += (float)s;
  } else {
    if (db2) db2[col - 2 * C - CO * C] += (float)s;
  }
}

// dy = gamma*invstd*(g - sum_g/count - xhat*sum_gxhat/count); partial rows [block][C]
// of sum_p dy (the wide conv's bias gradient).
template <int CO, int U = 2>
__global__ __launch_bounds__(256) void head_out_bwd_apply_kernel(
    const float* __restrict__ y, Act yd, const float* __restrict__ save,
    const float* __restrict__ gamma, const float* __restrict__ w2,
    const float* __restrict__ dout, Act dod, const double* __restrict__ sums, double count,
    int64_t ppb, int rows, float* __restrict__ dy, Act dyd, float* __restrict__ part) {
  extern __shared__ float red[];  // [rows][C], then the dout rows [ppb][CO]
  const int C = (int)yd.c, c4 = (C + 3) >> 2;
  const int tid = threadIdx.x;
  const int64_t P = yd.n * yd.h * yd.w;
  const int64_t p0 = blockIdx.x * ppb;
  const int64_t p1 = p0 + ppb < P ? p0 + ppb : P;
  const int r = tid / c4, q = tid - r * c4, c = 4 * q;
  float* sd = red + rows * C;
  head_stage_dout<CO>(sd, dout, dod, p0, p1);
  __syncthreads();
  if (tid < rows * c4) {
    const HeadCoef hc = head_coef(save, c, C);
    const float inv_n = (float)(1.0 / count);
    f4 wv[CO], mg, mgx, k4;
#pragma unroll
    for (int o = 0; o < CO; ++o) wv[o] = hchan4(w2 + (int64_t)o * C, c, C);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int ch = c + k < C ? c + k : C - 1;
      mg[k] = (float)sums[ch] * inv_n;
      mgx[k] = (float)sums[C + ch] * inv_n;
      k4[k] = (gamma ? gamma[ch] : 1.f) * hc.invstd[k];
    }
    f4 sdy = {0.f, 0.f, 0.f, 0.f};
    // U pixels in flight per thread
    // the next U pixels' y loads go out before this group's dy stores (vmcnt counts
    // stores too: loads issued after them would wait for them)
    f4 nv[U];
    auto ldy = [&](int64_t pb) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t p = pb + u * rows;
        nv[u] = p < p1 ? hld4(yb_at(y, P, p, c)) : f4{0.f, 0.f, 0.f, 0.f};
      }
    };
    ldy(p0 + r);
    for (int64_t pb = p0 + r; pb < p1; pb += U * rows) {
      f4 vv[U];
      float dd[U][CO];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t p = pb + u * rows;
        const bool ok = p < p1;
        vv[u] = nv[u];
#pragma unroll
        for (int o = 0; o < CO; ++o) dd[u][o] = ok ? sd[(p - p0) * CO + o] : 0.f;
      }
      if (pb + U * rows < p1) ldy(pb + U * rows);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t p = pb + u * rows;
        if (p >= p1) break;
        const f4 v = vv[u];
        f4 o4;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float h = __builtin_fmaf(v[k], hc.sc[k], hc.sh[k]);
          float dh = 0.f;
#pragma unroll
          for (int o = 0; o < CO; ++o) dh += wv[o][k] * dd[u][o];
          const float g = h > 0.f ? dh : 0.f;
          const float xh = (v[k] - hc.mean[k]) * hc.invstd[k];
          o4[k] = k4[k] * (g - mg[k] - xh * mgx[k]);
          sdy[k] += o4[k];
        }
        float* dst = dy + p * dyd.ps + c;
        if (c + 4 <= C) {
          *reinterpret_cast<f4*>(dst) = o4;
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (c + k < C) dst[k] = o4[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c + k < C) red[r * C + c + k] = sdy[k];
  }
  __syncthreads();
  for (int ch = tid; ch < C; ch += 256) {
    float a = 0.f;
    for (int i = 0; i < rows; ++i) a += red[i * C + ch];
    part[(int64_t)blockIdx.x * C + ch] = a;
  }
}

// ------------------------------------------------------------------ up-sum ----
// y[n,oy,x,c] = sum_k x0[n,oy,x,k] W0[c][k] + sum_s up(z_s)[n,oy,x,c] + bias[c]
// (the wide head conv split by branch; z_s = W_s y_s at the branch resolution).
// Workgroup = (band of kUsRows image rows, 64-pixel chunk, 64-channel block); wave w
// owns pixels 16w..16w+15 of each row.  The W0 fragments and the horizontal
// interpolation tables are set up once per workgroup; per row the full-resolution block
// W0 x0 (K = Cin0 <= 32) is a 16x64 MFMA tile per wave (v_mfma_f32_16x16x4f32), each
// source's two contributing rows are blended vertically into LDS (one batch of
// unconditional buffer loads, source columns clamped into the chunk's window), and the
// epilogue adds the two horizontal taps per source and the bias, stores y and
// accumulates the BN partial sums (written once per workgroup).
constexpr int kUsXB = 64, kUsCB = 64, kUsMaxCin = 32;
// LDS column stride of source s's blended row: the epilogue's 4 lane groups read columns
// 2 (s = 0), 1 (s = 1) or 0-1 (s = 2) apart, so stride * step = 16 (mod 32) puts each
// 32-lane half of a ds_read_b32 on distinct banks.
__host__ __device__ constexpr int us_vs(int s) { return s == 0 ? 72 : 80; }
constexpr int kUsRows = 8;                                          // image rows per workgroup

struct UpSum {
  const float* x;
  int x_ps, cin, cin4, H, W;
  uint32_t x_bytes;
  const float* wp;  // packed [round_up(C,64)][cin4]
  uint32_t wp_bytes;
  const float* bias;
  const float* z[3];
  uint32_t z_bytes[3];
  int zh[3], zw[3], zps[3];
  float sh[3], sw[3];
  int vcols[3];  // staged source columns per 64-pixel chunk
  float* y;
  uint32_t y_bytes;
  int C;
  float* stats;  // [2][rows][C], row = (n*nrb + band)*nxb + xb
  int rows, nxb, nrb;
};

// TIGHT: source s stages at most 4 * (12 >> s) columns per chunk (true for the HRNet
// heads, whose sources halve in resolution): 42 instead of 72 load / blend registers,
// so 3 instead of 2 waves per SIMD, and no clamped duplicate loads.
__host__ __device__ constexpr int us_vu(int s, bool tight) { return tight ? (12 >> s) : 12; }

// KQ: K quads of the W0 block held in registers (5 for Cin0 <= 20, the W18 heads'
// 18-channel branch; 8 up to kUsMaxCin): fewer fragment registers, 4 waves per SIMD.
template <int NUP, bool TIGHT, int KQ>
__global__ __launch_bounds__(256) void upsum_kernel(UpSum p) {
  extern __shared__ __attribute__((aligned(16))) float usm[];
  __shared__ double red[2][4][kUsCB];
  f4* tab = reinterpret_cast<f4*>(usm);                  // [NUP][kUsXB] {i0, i1, l0, l1}
  float* vs = usm + 4 * (NUP > 0 ? NUP : 1) * kUsXB;     // per source [vcols_s][us_vs(s)]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, r = lane & 15;
  // block order: chunk fastest, then channel block, then row band
  const int ncb = (p.C + kUsCB - 1) / kUsCB;
  const int xb = blockIdx.x % p.nxb, x0 = xb * kUsXB;
  const int cbi = (blockIdx.x / p.nxb) % ncb;
  const int band = blockIdx.x / (p.nxb * ncb);
  const int n = band / p.nrb, oy0 = (band - n * p.nrb) * kUsRows;
  const int ny = p.H - oy0 < kUsRows ? p.H - oy0 : kUsRows;
  const int c0 = cbi * kUsCB;
  const int xn = p.W - x0 < kUsXB ? p.W - x0 : kUsXB;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(p.wp, p.wp_bytes);
  const __amdgpu_buffer_rsrc_t yr = make_rsrc(p.y, p.y_bytes);
  // ---- W0 fragments (once) ----
  const int kq = p.cin4 >> 2;
  float fb[KQ][4];
#pragma unroll
  for (int kb = 0; kb < KQ; ++kb)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      fb[kb][j] = load1(wr, kb < kq ? (uint32_t)((c0 + 16 * j + r) * p.cin4 + 4 * kb + g) * 4u
                                    : kOOB);
  // ---- horizontal tables and source windows (once) ----
  const int c = c0 + lane;
  const bool cok = c < p.C;
  int vlo[3] = {0, 0, 0}, vhi[3] = {0, 0, 0}, voff[3] = {0, 0, 0};
#pragma unroll
  for (int s = 0; s < NUP; ++s) {
    vlo[s] = lerp_index(x0, p.zw[s], p.sw[s]).i0;
    vhi[s] = lerp_index(x0 + xn - 1, p.zw[s], p.sw[s]).i1;
    voff[s] = s == 0 ? 0 : voff[s - 1] + p.vcols[s - 1] * us_vs(s - 1);  // floats
    if (threadIdx.x < xn) {
      const Lerp lx = lerp_index(x0 + threadIdx.x, p.zw[s], p.sw[s]);
      tab[s * kUsXB + threadIdx.x] =
          f4{__int_as_float(voff[s] + (lx.i0 - vlo[s]) * us_vs(s)),
             __int_as_float(voff[s] + (lx.i1 - vlo[s]) * us_vs(s)), lx.l0, lx.l1};
    }
  }
  float bj[4];
  double s1[4], s2[4];  // BN partial sums over the band (per-row float sums added in double)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cj = c0 + 16 * j + r;
    bj[j] = (p.bias && cj < p.C) ? p.bias[cj] : 0.f;
    s1[j] = 0.0;
    s2[j] = 0.0;
  }
  const int64_t P = (int64_t)(p.rows / p.nxb / p.nrb) * p.H * p.W;  // n * H * W
  constexpr int VU = 12;  // source columns per wave (host: vcols_s <= 4 * us_vu(s, TIGHT))
  const int pxa = 16 * wave + r;
  for (int ry = 0; ry < ny; ++ry) {
    const int oy = oy0 + ry, row = n * p.H + oy;
    // ---- loads: x0 fragments and the two source rows of every source ----
    float fa[KQ];
#pragma unroll
    for (int kb = 0; kb < KQ; ++kb) {
      const int k = 4 * kb + g;
      fa[kb] = load1(xr, (kb < kq && pxa < xn && k < p.cin)
                             ? (uint32_t)(((row * p.W + x0 + pxa) * p.x_ps + k) * 4u) : kOOB);
    }
    float a0[NUP > 0 ? NUP : 1][VU], a1[NUP > 0 ? NUP : 1][VU];  // only [s][< us_vu] live
    Lerp ly[3];
#pragma unroll
    for (int s = 0; s < NUP; ++s) {
      ly[s] = lerp_index(oy, p.zh[s], p.sh[s]);
      const __amdgpu_buffer_rsrc_t zr = make_rsrc(p.z[s], p.z_bytes[s]);
      const int rb0 = ((n * p.zh[s] + ly[s].i0) * p.zw[s]) * p.zps[s] + c;
      const int rb1 = ((n * p.zh[s] + ly[s].i1) * p.zw[s]) * p.zps[s] + c;
#pragma unroll
      for (int u = 0; u < us_vu(s, TIGHT); ++u) {
        int ix = vlo[s] + wave + 4 * u;
        ix = ix < vhi[s] ? ix : vhi[s];
        a0[s][u] = load1(zr, cok ? (uint32_t)(rb0 + ix * p.zps[s]) * 4u : kOOB);
        a1[s][u] = load1(zr, cok ? (uint32_t)(rb1 + ix * p.zps[s]) * 4u : kOOB);
      }
    }
    __syncthreads();  // the previous row's epilogue reads of vs are done (and tab is written)
#pragma unroll
    for (int s = 0; s < NUP; ++s) {
#pragma unroll
      for (int u = 0; u < us_vu(s, TIGHT); ++u) {
        const int j = wave + 4 * u;  // uniform per wave
        if (vlo[s] + j <= vhi[s])
          vs[voff[s] + j * us_vs(s) + lane] = ly[s].l0 * a0[s][u] + ly[s].l1 * a1[s][u];
      }
    }
    // ---- W0 x0: acc[j][e] = pixel 16*wave + 4g + e, channel c0 + 16j + r ----
    f4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KQ; ++kb) {
      if (kb < kq) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[kb], fb[kb][j], acc[j], 0, 0, 0);
      }
    }
    __syncthreads();
    // ---- epilogue ----
    const uint32_t ybase = (uint32_t)(cbi * P * 64 + ((int64_t)row * p.W + x0) * 64 + r);
    float r1[4] = {0.f, 0.f, 0.f, 0.f}, r2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int px = 16 * wave + 4 * g + e;
      f4 t[3];
#pragma unroll
      for (int s = 0; s < NUP; ++s) t[s] = tab[s * kUsXB + (px < xn ? px : xn - 1)];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = acc[j][e];
#pragma unroll
        for (int s = 0; s < NUP; ++s) {
          const float* vj = vs + 16 * j + r;
          v += t[s][2] * vj[__float_as_int(t[s][0])] + t[s][3] * vj[__float_as_int(t[s][1])];
        }
        const bool ok = px < xn && c0 + 16 * j + r < p.C;
        store1(yr, ok ? (ybase + px * 64 + 16 * j) * 4u : kOOB, v + bj[j]);
        r1[j] += ok ? v : 0.f;  // statistics of y - bias (shifted)
        r2[j] += ok ? v * v : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s1[j] += (double)r1[j];
      s2[j] += (double)r2[j];
    }
  }
  if (p.stats) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s1[j] += __shfl_xor(s1[j], 16, 64);
      s1[j] += __shfl_xor(s1[j], 32, 64);
      s2[j] += __shfl_xor(s2[j], 16, 64);
      s2[j] += __shfl_xor(s2[j], 32, 64);
    }
    if (g == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        red[0][wave][16 * j + r] = s1[j];
        red[1][wave][16 * j + r] = s2[j];
      }
    }
    __syncthreads();
    if (wave == 0 && cok) {
      const int rr = (n * p.nrb + oy0 / kUsRows) * p.nxb + xb;
      p.stats[(int64_t)rr * p.C + c] =
          (float)(red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane]);
      p.stats[((int64_t)p.rows + rr) * p.C + c] =
          (float)(red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane]);
    }
  }
}

// One-pass up-sum for exact 2^(s+1) sources (the HRNet heads' branches halve in size):
// lane = channel, wave w owns pixels [x0 + 16w, x0 + 16w + 16) of the workgroup's kUsRows
// rows, so nothing is staged in LDS and no barrier runs before the statistics.  W0 x0 is
// computed on the VALU (K = Cin0 <= 4*KQ, 2.6 GF per head: ~10 us of VALU chip-wide) with the
// x0 pixel -- uniform over the lanes -- in scalar registers (constant-address-space loads);
// each source keeps its two rows of the wave's 16/F + 2 source columns in registers,
// re-loaded only when the row pair moves (a row is loaded once per workgroup); the bilinear
// weights are exact (integer arithmetic on pow2 ratios, compile-time horizontally).  Same
// output layout (B64) and statistics rows (y - bias) as upsum_kernel.
__host__ __device__ constexpr int us2_off(int pp, int F) {  // floor((pp + 0.5) / F - 0.5)
  return 2 * pp + 1 - F >= 0 ? (2 * pp + 1 - F) / (2 * F) : -1;
}
__host__ __device__ constexpr float us2_frac(int pp, int F) {
  return (float)(2 * pp + 1 - F - 2 * F * us2_off(pp, F)) / (float)(2 * F);
}

template <int S>
struct Us2Src {
  static constexpr int F = 2 << S, NC = 16 / F + 2;  // source columns px0/F - 1 ... px0/F + 16/F
  float r0[NC], r1[NC];
  int h0, h1;      // rows held in r0 / r1
  float l0, l1;    // vertical weights of the row they serve
};

template <int S>
__device__ __forceinline__ void us2_rows(Us2Src<S>& a, const UpSum& p, int n, int oy, int px0,
                                         int c, bool cok) {
  constexpr int F = Us2Src<S>::F, NC = Us2Src<S>::NC;
  const int num = 2 * oy + 1 - F;
  const int i0 = num >= 0 ? num / (2 * F) : -1;
  a.l1 = (float)(num - 2 * F * i0) / (float)(2 * F);
  a.l0 = 1.f - a.l1;
  const int zh = p.zh[S], zw = p.zw[S];
  const int ra = i0 < 0 ? 0 : (i0 > zh - 1 ? zh - 1 : i0);
  const int rb = i0 + 1 > zh - 1 ? zh - 1 : i0 + 1;
  if (ra == a.h0 && rb == a.h1) return;
  const __amdgpu_buffer_rsrc_t zr = make_rsrc(p.z[S], p.z_bytes[S]);
  const int cb = px0 / F - 1;
  auto load = [&](int row, float* dst) {
    const int rbase = (n * zh + row) * zw;
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      int col = cb + q;
      col = col < 0 ? 0 : (col > zw - 1 ? zw - 1 : col);
      dst[q] = load1(zr, cok ? (uint32_t)((rbase + col) * p.zps[S] + c) * 4u : kOOB);
    }
  };
  if (ra == a.h1) {
#pragma unroll
    for (int q = 0; q < NC; ++q) a.r0[q] = a.r1[q];
  } else {
    load(ra, a.r0);
  }
  if (rb != a.h1) load(rb, a.r1);
  a.h0 = ra;
  a.h1 = rb;
}

template <int S>
__device__ __forceinline__ void us2_add(const Us2Src<S>& a, float* v) {
  constexpr int F = Us2Src<S>::F, NC = Us2Src<S>::NC;
  float vb[NC];
#pragma unroll
  for (int q = 0; q < NC; ++q) vb[q] = a.l0 * a.r0[q] + a.l1 * a.r1[q];
#pragma unroll
  for (int pp = 0; pp < 16; ++pp) {
    const int o = us2_off(pp, F) + 1;
    const float h1 = us2_frac(pp, F), h0 = 1.f - us2_frac(pp, F);
    v[pp] += h0 * vb[o] + h1 * vb[o + 1];
  }
}

template <int NUP, int KQ>
__global__ __launch_bounds__(256) void upsum2_kernel(UpSum p) {
  __shared__ double red[2][4][kUsCB];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ncb = (p.C + kUsCB - 1) / kUsCB;
  const int xb = blockIdx.x % p.nxb, x0 = xb * kUsXB;
  const int cbi = (blockIdx.x / p.nxb) % ncb;
  const int band = blockIdx.x / (p.nxb * ncb);
  const int n = band / p.nrb, oy0 = (band - n * p.nrb) * kUsRows;
  const int ny = p.H - oy0 < kUsRows ? p.H - oy0 : kUsRows;
  const int c = cbi * kUsCB + lane;
  const bool cok = c < p.C;
  const int px0 = x0 + 16 * wave;
  const int g = lane >> 4, r = lane & 15;
  // W0 fragments: B[k = 4kq + g][n = 16j + r] of the channel block (packed, zero padded)
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(p.wp, p.wp_bytes);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  float fb[KQ][4];
#pragma unroll
  for (int kq = 0; kq < KQ; ++kq)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      fb[kq][j] = load1(wr, (uint32_t)((cbi * kUsCB + 16 * j + r) * p.cin4 + 4 * kq + g) * 4u);
  __shared__ float xts[4][16 * 64];
  float* xt = xts[wave];
  const float bias = (p.bias && cok) ? p.bias[c] : 0.f;
  Us2Src<0> s0;
  Us2Src<1> s1;
  Us2Src<2> s2;
  s0.h0 = s0.h1 = s1.h0 = s1.h1 = s2.h0 = s2.h1 = -1;
  const __amdgpu_buffer_rsrc_t yr = make_rsrc(p.y, p.y_bytes);
  const int64_t P = (int64_t)(p.rows / p.nxb / p.nrb) * p.H * p.W;  // n * H * W
  double d1 = 0.0, d2 = 0.0;
  // Row ry + 1's loads (x0 fragments, source rows that move) are issued before row ry's
  // stores: vmcnt counts stores too, so a load issued after them would wait for them.
  float xa[KQ];
  auto prep = [&](int oy) {
    const int row = n * p.H + oy;
    const uint32_t xo = (uint32_t)(((row * p.W + px0 + r) * p.x_ps + g) * 4);
#pragma unroll
    for (int kq = 0; kq < KQ; ++kq) xa[kq] = load1(xr, 4 * kq + g < p.cin ? xo + 16u * kq : kOOB);
    if constexpr (NUP > 0) us2_rows<0>(s0, p, n, oy, px0, c, cok);
    if constexpr (NUP > 1) us2_rows<1>(s1, p, n, oy, px0, c, cok);
    if constexpr (NUP > 2) us2_rows<2>(s2, p, n, oy, px0, c, cok);
  };
  prep(oy0);
  for (int ry = 0; ry < ny; ++ry) {
    const int oy = oy0 + ry, row = n * p.H + oy;
    float v[16];
    {  // W0 x0 on MFMA (A = x0[px][k], B = W0 fragments), through this wave's LDS tile
       // to lane = channel: lane (g, r) holds channels 16j + r of pixels 4g + e
      f4 acc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kq = 0; kq < KQ; ++kq)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[kq], fb[kq][j], acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) xt[(4 * g + e) * 64 + 16 * j + r] = acc[j][e];
#pragma unroll
      for (int pp = 0; pp < 16; ++pp) v[pp] = xt[pp * 64 + lane];
    }
    if constexpr (NUP > 0) us2_add<0>(s0, v);
    if constexpr (NUP > 1) us2_add<1>(s1, v);
    if constexpr (NUP > 2) us2_add<2>(s2, v);
    if (ry + 1 < ny) prep(oy + 1);
    const uint32_t ybase = (uint32_t)(cbi * P * 64 + ((int64_t)row * p.W + px0) * 64 + lane);
    float q1 = 0.f, q2 = 0.f;
#pragma unroll
    for (int pp = 0; pp < 16; ++pp) {
      store1(yr, cok ? (ybase + pp * 64) * 4u : kOOB, v[pp] + bias);
      q1 += v[pp];
      q2 += v[pp] * v[pp];
    }
    d1 += (double)q1;
    d2 += (double)q2;
  }
  if (p.stats) {
    red[0][wave][lane] = d1;
    red[1][wave][lane] = d2;
    __syncthreads();
    if (wave == 0 && cok) {
      const int rr = (n * p.nrb + oy0 / kUsRows) * p.nxb + xb;
      p.stats[(int64_t)rr * p.C + c] =
          (float)(red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane]);
      p.stats[((int64_t)p.rows + rr) * p.C + c] =
          (float)(red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane]);
    }
  }
}

// ------------------------------------------- upsampling adjoint, all sources ----
// dx_s = up_s^T(dy) for every source s at once, separably.
// Horizontal pass, workgroup = (dY row, 64-pixel chunk, 64-channel block): source
// columns are partitioned between chunks (ix belongs to the chunk holding the output
// coordinate of its centre), the chunk's dY pixels plus the interpolation halo are
// staged in LDS once with per-pixel forward tables {i0, i1, l0, l1}, and each owned
// column gathers hb_s[n][oy][ix][c] = sum_ox w(ox, ix) dy[n][oy][ox][c] from LDS.
// Vertical pass, workgroup = (target row, 64-channel block): the row's weights are
// tabulated once, then dx_s[n][iy][ix][c] = sum_oy w(oy, iy) hb_s[n][oy][ix][c].
// The weights are exactly upsample_fwd_kernel's (lerp_index).  Lane = channel.
struct UpAdj {
  const float* dy;
  int dy_ps, H, W, C;
  float* hb[3];
  float* dx[3];
  int zh[3], zw[3], dx_ps[3];
  float sh[3], sw[3];
  int halo, nxb;
  float beta[3];  // up_adj3_kernel: dx_s = adjoint + beta_s * dx_s (the fuse adjoints)
};

__device__ __forceinline__ void adj_window(int i, int in_size, int out_size, float scale,
                                           int& lo, int& hi) {
  lo = (int)floorf(((float)i - 0.5f) / scale - 0.5f) - 1;
  hi = (int)ceilf(((float)i + 1.5f) / scale - 0.5f) + 1;
  if (lo < 0) lo = 0;
  if (hi > out_size - 1) hi = out_size - 1;
  if (i == in_size - 1) hi = out_size - 1;  // clamped sources beyond the last input
}

// First source column owned by chunk xb (monotone in xb; xb = nxb gives zw).
__device__ __forceinline__ int adj_owned_begin(int xb, int nxb, int zw, float sw) {
  if (xb >= nxb) return zw;
  if (xb <= 0) return 0;
  int b = (int)ceilf(((float)(xb * kUsXB) + 0.5f) * sw - 0.5f);
  return b < 0 ? 0 : (b > zw ? zw : b);
}

template <int NUP>
__global__ __launch_bounds__(256) void up_adj_h_kernel(UpAdj p) {
  extern __shared__ __attribute__((aligned(16))) float asm_[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ncb = (p.C + 63) / 64;
  const int xb = blockIdx.x % p.nxb;
  const int cbi = (blockIdx.x / p.nxb) % ncb;
  const int row = blockIdx.x / (p.nxb * ncb);  // n*H + oy
  const int span = kUsXB + 2 * p.halo;
  f4* tab = reinterpret_cast<f4*>(asm_);              // [NUP][span]
  float* st = asm_ + 4 * NUP * span;                  // [span][64]
  int ib[3], ie[3], wlo = 1 << 30, whi = -1;
#pragma unroll
  for (int s = 0; s < NUP; ++s) {
    ib[s] = adj_owned_begin(xb, p.nxb, p.zw[s], p.sw[s]);
    ie[s] = adj_owned_begin(xb + 1, p.nxb, p.zw[s], p.sw[s]);
    if (ie[s] > ib[s]) {
      int lo, hi, lo2, hi2;
      adj_window(ib[s], p.zw[s], p.W, p.sw[s], lo, hi);
      adj_window(ie[s] - 1, p.zw[s], p.W, p.sw[s], lo2, hi2);
      wlo = lo < wlo ? lo : wlo;
      whi = hi2 > whi ? hi2 : whi;
    }
  }
  if (whi < wlo) return;  // no owned columns (uniform over the workgroup)
  const int cnt = whi - wlo + 1;  // <= span (host-sized halo)
#pragma unroll
  for (int s = 0; s < NUP; ++s) {
    for (int i = threadIdx.x; i < cnt; i += 256) {
      const Lerp lx = lerp_index(wlo + i, p.zw[s], p.sw[s]);
      tab[s * span + i] = f4{__int_as_float(lx.i0), __int_as_float(lx.i1), lx.l0, lx.l1};
    }
  }
  {
    const int c = cbi * 64 + lane;
    const bool cok = c < p.C;
    const float* drow = p.dy + (int64_t)row * p.W * p.dy_ps + c;
    {
      constexpr int SU = 24;  // pixels per wave in flight (span <= 96: one round trip)
      for (int i0 = wave; i0 < cnt; i0 += 4 * SU) {
        float v[SU];
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int i = i0 + 4 * u;
          v[u] = (cok && i < cnt) ? drow[(int64_t)(wlo + i) * p.dy_ps] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int i = i0 + 4 * u;
          if (i < cnt) st[i * 64 + lane] = v[u];
        }
      }
    }
    __syncthreads();
    if (!cok) return;
    // Work items: (source, half of its owned columns); wave w streams items w, w+4, ...
    // Streaming: pixels ox ascend, so each ox adds l0 to column i0 and l1 to i1 in
    // {i0, i0+1} with i0 non-decreasing; two running sums (columns cur, cur+1) are kept
    // and column cur is final (stored) once i0 moves past it.
    for (int item = wave; item < 2 * NUP; item += 4) {
      const int s = item % NUP, half = item / NUP;
      const int mid = ib[s] + (ie[s] - ib[s] + 1) / 2;
      const int cb = half ? mid : ib[s], ce = half ? ie[s] : mid;
      if (cb >= ce) continue;
      int lo, hi, lo2, hi2;
      adj_window(cb, p.zw[s], p.W, p.sw[s], lo, hi);
      adj_window(ce - 1, p.zw[s], p.W, p.sw[s], lo2, hi2);
      float* hrow = p.hb[s] + (int64_t)row * p.zw[s] * p.C + c;
      const f4* ts = tab + s * span - wlo;
      const float* sv = st - wlo * 64 + lane;
      int cur = cb - 1;
      float a0 = 0.f, a1 = 0.f;  // sums of columns cur, cur + 1
      for (int ox = lo; ox <= hi2; ++ox) {
        const f4 t = ts[ox];  // wave-uniform: moved to scalar registers
        const int i0 = __builtin_amdgcn_readfirstlane(__float_as_int(t[0]));
        const int i1 = __builtin_amdgcn_readfirstlane(__float_as_int(t[1]));
        const float l0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(t[2])));
        const float l1 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(t[3])));
        const float v = sv[ox * 64];
        while (cur < i0) {  // wave-uniform
          if (cur >= cb && cur < ce) hrow[(int64_t)cur * p.C] = a0;
          a0 = a1;
          a1 = 0.f;
          ++cur;
        }
        // now i0 <= cur (i0 < cur only left of the owned range: not ours)
        if (i0 == cur) a0 = __builtin_fmaf(l0, v, a0);
        if (i1 == cur) a0 = __builtin_fmaf(l1, v, a0);
        else if (i1 == cur + 1) a1 = __builtin_fmaf(l1, v, a1);
      }
      if (cur >= cb && cur < ce) hrow[(int64_t)cur * p.C] = a0;
      if (cur + 1 >= cb && cur + 1 < ce) hrow[(int64_t)(cur + 1) * p.C] = a1;
    }
  }
}

__global__ __launch_bounds__(256) void up_adj_v_kernel(UpAdj p, int s) {
  __shared__ float wy[64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = blockIdx.x;  // n*zh + iy
  const int n = row / p.zh[s], iy = row - n * p.zh[s];
  const int c = blockIdx.y * 64 + lane;
  int lo, hi;
  adj_window(iy, p.zh[s], p.H, p.sh[s], lo, hi);
  const int cnt = hi - lo + 1 < 64 ? hi - lo + 1 : 64;  // host guarantees <= 64
  if (threadIdx.x < cnt) {
    const Lerp ly = lerp_index(lo + threadIdx.x, p.zh[s], p.sh[s]);
    wy[threadIdx.x] = (ly.i0 == iy ? ly.l0 : 0.f) + (ly.i1 == iy ? ly.l1 : 0.f);
  }
  __syncthreads();
  if (c >= p.C) return;
  const float* hb = p.hb[s] + ((int64_t)n * p.H + lo) * p.zw[s] * p.C + c;
  float* out = p.dx[s] + (int64_t)row * p.zw[s] * p.dx_ps[s] + c;
  const int64_t rs = (int64_t)p.zw[s] * p.C;
  for (int ix = wave; ix < p.zw[s]; ix += 8) {
    const bool two = ix + 4 < p.zw[s];
    const float* h0 = hb + (int64_t)ix * p.C;
    const float* h1 = hb + (int64_t)(two ? ix + 4 : ix) * p.C;
    float acc0 = 0.f, acc1 = 0.f;
#pragma unroll 4
    for (int t = 0; t < cnt; ++t) {
      acc0 = __builtin_fmaf(wy[t], h0[t * rs], acc0);
      acc1 = __builtin_fmaf(wy[t], h1[t * rs], acc1);
    }
    out[(int64_t)ix * p.dx_ps[s]] = acc0;
    if (two) out[(int64_t)(ix + 4) * p.dx_ps[s]] = acc1;
  }
}

// Exact 2^(s+1) ratios: static stencils (hat_w, common.h).
constexpr int kAdjHalo = 4;  // F/2 for F <= 8

// Horizontal pass, workgroup = (dY row, 64-pixel chunk, 64-channel block); the chunk and a
// 4-pixel halo are staged in LDS (lane = channel); wave w computes the owned source
// columns j = w, w + 4, ... of every source with immediate LDS offsets.
template <int NUP>
__global__ __launch_bounds__(256) void up_adj2_h_kernel(UpAdj p) {
  constexpr int SPAN = kUsXB + 2 * kAdjHalo, PER = SPAN / 4;
  __shared__ float st[SPAN][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ncb = (p.C + 63) / 64;
  const int xb = blockIdx.x % p.nxb;
  const int cbi = (blockIdx.x / p.nxb) % ncb;
  const int row = blockIdx.x / (p.nxb * ncb);  // n*H + oy
  const int c = cbi * 64 + lane;
  const bool cok = c < p.C;
  const int x0 = xb * kUsXB;
  const float* drow = p.dy + (int64_t)row * p.W * p.dy_ps + (cok ? c : 0);
  float v[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int ox = x0 - kAdjHalo + wave + 4 * u;
    v[u] = (cok && ox >= 0 && ox < p.W) ? drow[(int64_t)ox * p.dy_ps] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) st[wave + 4 * u][lane] = v[u];
  __syncthreads();
  if (!cok) return;
#pragma unroll
  for (int s = 0; s < NUP; ++s) {
    const int F = 2 << s, zw = p.zw[s];
    const float* sw = &st[F * wave + kAdjHalo][lane];  // column j = wave: pixels F*wave + d
    float* hrow = p.hb[s] + (int64_t)row * zw * p.C + c;
#pragma unroll
    for (int jj = 0; jj < kUsXB / (2 << s) / 4; ++jj) {
      const int j = wave + 4 * jj, ix = x0 / F + j;
      float acc = 0.f;
#pragma unroll
      for (int d = -(1 << s); d < 3 * (1 << s); ++d) acc += hat_w(d, F) * sw[(4 * F * jj + d) * 64];
      if (ix == 0) {  // virtual column -1 (pixels d - F)
#pragma unroll
        for (int d = 2 << s; d < 3 * (1 << s); ++d) acc += hat_w(d, F) * sw[(d - F) * 64];
      }
      if (ix == zw - 1) {  // virtual column zw (pixels F*(j+1) + d)
#pragma unroll
        for (int d = -(1 << s); d < 0; ++d) acc += hat_w(d, F) * sw[(4 * F * jj + F + d) * 64];
      }
      hrow[(int64_t)ix * p.C] = acc;
    }
  }
}

// Vertical pass of source S (F = 2^(S+1)), workgroup = (target row, 64-channel block).
template <int S>
__global__ __launch_bounds__(256) void up_adj2_v_kernel(UpAdj p) {
  constexpr int F = 2 << S, HF = 1 << S;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row = blockIdx.x;  // n*zh + iy
  const int zh = p.zh[S], zw = p.zw[S];
  const int n = row / zh, iy = row - n * zh;
  const int c = blockIdx.y * 64 + lane;
  if (c >= p.C) return;
  const int64_t rs = (int64_t)zw * p.C;
  const float* hb = p.hb[S] + (int64_t)n * p.H * rs + c;
  float* out = p.dx[S] + (int64_t)row * zw * p.dx_ps[S] + c;
  const int oy0 = F * iy;
  constexpr int U = 4;  // target columns per wave iteration (their loads in flight together)
  constexpr int NT = 3 * F;  // 2F taps + the two edge folds (HF rows each)
  for (int ix0 = wave; ix0 < zw; ix0 += 4 * U) {
    float v[U][NT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ix = ix0 + 4 * u;
      const float* h = hb + (int64_t)(ix < zw ? ix : zw - 1) * p.C;
#pragma unroll
      for (int d = -HF; d < 3 * HF; ++d) {
        const int oy = oy0 + d;
        v[u][d + HF] = (oy >= 0 && oy < p.H) ? h[(int64_t)oy * rs] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < HF; ++e) {  // edge folds: rows d - F (top, d = F + e), F*zh + d
        v[u][2 * F + e] = iy == 0 ? h[(int64_t)e * rs] : 0.f;
        v[u][2 * F + HF + e] = iy == zh - 1 ? h[(int64_t)(F * zh - HF + e) * rs] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ix = ix0 + 4 * u;
      if (ix >= zw) break;
      float acc = 0.f;
#pragma unroll
      for (int d = -HF; d < 3 * HF; ++d) acc += hat_w(d, F) * v[u][d + HF];
      if (iy == 0) {
#pragma unroll
        for (int e = 0; e < HF; ++e) acc += hat_w(F + e, F) * v[u][2 * F + e];
      }
      if (iy == zh - 1) {
#pragma unroll
        for (int e = 0; e < HF; ++e) acc += hat_w(e - HF, F) * v[u][2 * F + HF + e];
      }
      out[(int64_t)ix * p.dx_ps[S]] = acc;
    }
  }
}

// Streaming form of the vertical pass: it only mixes hb rows, and an hb row
// (zw * C floats, ix-major) is contiguous, so thread = 4 consecutive floats of the row:
// one 16-byte load per contributing row (2F taps, plus the edge folds on the first / last
// target row: uniform per workgroup), the same weights and summation order as
// up_adj2_v_kernel, then the 4 results go to (ix, c) = divmod(k, C) of the (possibly
// channel-padded) dx layout.  Workgroup = (target row, slice of the row).  Needs
// zw * C % 4 == 0 (16-byte aligned rows).
static int g_adj_stream = 1;  // vae2_heads_set_algo bit 0 clears it
static int g_upsum_tight = 1;  // vae2_heads_set_algo bit 1 clears it
static int g_upsum_one = 1;    // vae2_heads_set_algo bit 3 clears it (upsum2_kernel)
// vae2_heads_set_algo bit 6 sets it: the fuse adjoints (resample.hip) through the one-pass
// band kernel -- off: with 18-72 channels a 64-lane channel block is mostly idle and the
// step measured 851-853 vs 861-866 frames/s through the two-pass quad kernels (A/B, same box)
int g_fuse_adj3 = 0;
int g_relu_dual_q = 1;         // vae2_heads_set_algo bit 7 clears it (relu_bwd_dual quad form)
static int g_head_red_u = 2;   // vae2_heads_set_algo bit 4: 4 pixels in flight (backward reduce)
static int g_head_app_u = 2;   // vae2_heads_set_algo bit 5: 4 pixels in flight (backward apply)

template <int S>
__global__ __launch_bounds__(256) void up_adj2_vs_kernel(UpAdj p, FastDiv cdiv) {
  constexpr int F = 2 << S, HF = 1 << S;
  const int row = blockIdx.x;  // n*zh + iy
  const int zh = p.zh[S], zw = p.zw[S];
  const int n = row / zh, iy = row - n * zh;
  const int64_t rs = (int64_t)zw * p.C;
  const int nq = (int)(rs >> 2);
  const float* hb = p.hb[S] + (int64_t)n * p.H * rs;
  float* out = p.dx[S] + (int64_t)row * zw * p.dx_ps[S];
  const int oy0 = F * iy;
  const uint32_t C = (uint32_t)p.C, dps = (uint32_t)p.dx_ps[S];
  for (int q = blockIdx.y * 256 + threadIdx.x; q < nq; q += gridDim.y * 256) {
    const int64_t k4 = 4 * (int64_t)q;
    f4 v[4 * HF];
#pragma unroll
    for (int d = -HF; d < 3 * HF; ++d) {
      const int oy = oy0 + d;
      v[d + HF] = (oy >= 0 && oy < p.H) ? *reinterpret_cast<const f4*>(hb + oy * rs + k4)
                                        : f4{0.f, 0.f, 0.f, 0.f};
    }
    f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = -HF; d < 3 * HF; ++d) acc += hat_w(d, F) * v[d + HF];
    if (iy == 0) {
#pragma unroll
      for (int e = 0; e < HF; ++e)
        acc += hat_w(F + e, F) * *reinterpret_cast<const f4*>(hb + e * rs + k4);
    }
    if (iy == zh - 1) {
#pragma unroll
      for (int e = 0; e < HF; ++e)
        acc += hat_w(e - HF, F) *
               *reinterpret_cast<const f4*>(hb + (int64_t)(F * zh - HF + e) * rs + k4);
    }
    uint32_t ix = cdiv.div((uint32_t)k4), c = (uint32_t)k4 - ix * C;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      out[(int64_t)ix * dps + c] = acc[i];
      if (++c == C) { c = 0; ++ix; }
    }
  }
}

// One-pass form of the power-of-two adjoint: dx_s = V_s^T H_s^T dy for every source with
// dy read once (plus a row halo) and no hb intermediate (the two-pass form above writes and
// re-reads 1/2 + 1/4 + 1/8 of dy).  Workgroup = (image, band of `br` dy rows, 64-pixel
// chunk, 64-channel block); lane = channel; wave w owns the source columns whose pixels
// start in [x0 + 16w, x0 + 16w + 16): 16/F per source.  The band's dy rows plus HF_max rows
// above and below stream through registers (the next row's loads in flight during the
// current row's arithmetic).  A dy row oy feeds exactly two target rows of source s,
// ih = (oy + HF) / F and ih - 1 (taps d = oy - F*ih and d + F); per source and owned column
// two accumulators follow them, and a row is stored once oy has moved past it.  Virtual
// rows / columns -1 and z are folded into 0 / z-1 as in up_adj2_h / up_adj2_vs, with the
// same hat_w weights; interior outputs keep the two-pass summation order.
static int g_adj_fused = 1;  // vae2_heads_set_algo bit 2 clears it
static int g_adj_band = 32;  // dy rows per workgroup (a multiple of 8)

// Logical block order with consecutive ids on one XCD (the hardware deals workgroups out
// round-robin over the 8 XCDs): neighbouring chunks / bands share dy halo rows in that L2.
__device__ __forceinline__ int xcd_remap_blocks(int orig, int n) {
  const int q = n >> 3, rr = n & 7, x = orig & 7;
  return (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (orig >> 3);
}

// Per-source state of up_adj3_kernel: the wave's 16/F owned columns in the two target rows
// the current dy row feeds (lo = ih - 1, hi = ih), cur = ih.
template <int S>
struct Adj3Src {
  static constexpr int F = 2 << S, HF = 1 << S, J = 8 >> S;
  float lo[J], hi[J];
  int cur;
};

template <int S>
__device__ __forceinline__ void adj3_store(const Adj3Src<S>& a, const UpAdj& p, int n, int iy,
                                           int b0, int b1, int px0, int c, bool cok) {
  constexpr int F = Adj3Src<S>::F;
  if (!cok || iy < b0 / F || iy >= b1 / F) return;
  float* out = p.dx[S] + ((int64_t)n * p.zh[S] + iy) * p.zw[S] * p.dx_ps[S] + c;
  const int ix0 = px0 / F;
  const float beta = p.beta[S];
  if (beta != 0.f) {
    float old[Adj3Src<S>::J];
#pragma unroll
    for (int j = 0; j < Adj3Src<S>::J; ++j) old[j] = out[(int64_t)(ix0 + j) * p.dx_ps[S]];
#pragma unroll
    for (int j = 0; j < Adj3Src<S>::J; ++j)
      out[(int64_t)(ix0 + j) * p.dx_ps[S]] = a.lo[j] + beta * old[j];
    return;
  }
#pragma unroll
  for (int j = 0; j < Adj3Src<S>::J; ++j) out[(int64_t)(ix0 + j) * p.dx_ps[S]] = a.lo[j];
}

// dy row oy (pixels px0 - HM + i in v[i]) into source S's accumulators.
template <int S, int HM>
__device__ __forceinline__ void adj3_row(Adj3Src<S>& a, const float* v, int oy, const UpAdj& p,
                                         int n, int b0, int b1, int px0, int c, bool cok) {
  constexpr int F = Adj3Src<S>::F, HF = Adj3Src<S>::HF, J = Adj3Src<S>::J;
  const int ih = (oy + HF) >> (S + 1);
  if (ih != a.cur) {  // target row cur - 1 is complete
    adj3_store<S>(a, p, n, a.cur - 1, b0, b1, px0, c, cok);
#pragma unroll
    for (int j = 0; j < J; ++j) {
      a.lo[j] = a.hi[j];
      a.hi[j] = 0.f;
    }
    a.cur = ih;
  }
  const int d = oy - F * ih;
  const float wh = hat_w(d, F), wl = hat_w(d + F, F);
  const int zw = p.zw[S], ix0 = px0 / F;
  const int mode = ih == p.zh[S] ? 2 : ih == 0 ? 1 : 0;  // 2: row zh folds into zh - 1; 1: -1 into 0
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const float* vj = v + HM + F * j;  // pixel px0 + F*j
    float h = 0.f;
#pragma unroll
    for (int dd = -HF; dd < 3 * HF; ++dd) h += hat_w(dd, F) * vj[dd];
    if (ix0 + j == 0) {  // virtual column -1 (pixels dd - F)
#pragma unroll
      for (int dd = F; dd < 3 * HF; ++dd) h += hat_w(dd, F) * vj[dd - F];
    }
    if (ix0 + j == zw - 1) {  // virtual column zw (pixels F*(j+1) + dd)
#pragma unroll
      for (int dd = -HF; dd < 0; ++dd) h += hat_w(dd, F) * vj[F + dd];
    }
    if (mode == 2) {
      a.lo[j] += wh * h;
      a.lo[j] += wl * h;
    } else if (mode == 1) {
      a.hi[j] += wh * h;
      a.hi[j] += wl * h;
    } else {
      a.hi[j] += wh * h;
      a.lo[j] += wl * h;
    }
  }
}

template <int NUP>
__global__ __launch_bounds__(256) void up_adj3_kernel(UpAdj p, int br, int nband) {
  constexpr int HM = 1 << (NUP - 1);  // row / pixel halo: HF of the coarsest source
  constexpr int NV = 16 + 2 * HM;     // dy pixels per wave and row
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ncb = (p.C + 63) >> 6;
  const int lb = xcd_remap_blocks(blockIdx.x, gridDim.x);
  const int xb = lb % p.nxb;
  int t = lb / p.nxb;
  const int cbi = t % ncb;
  t /= ncb;
  const int band = t % nband, n = t / nband;
  const int c = cbi * 64 + lane;
  const bool cok = c < p.C;
  const int b0 = band * br, b1 = b0 + br < p.H ? b0 + br : p.H;
  const int ys = b0 - HM > 0 ? b0 - HM : 0, ye = b1 + HM < p.H ? b1 + HM : p.H;
  const int px0 = xb * kUsXB + 16 * wave;
  // One buffer resource per dy row (num_records = the row's bytes): pixels left of the row
  // wrap to huge offsets and pixels right of it exceed the row, so both load 0 with no
  // per-pixel test; pad channels use an offset past any row.
  const uint32_t pstep = (uint32_t)p.dy_ps * 4u, rbytes = (uint32_t)p.W * pstep;
  const uint32_t loff = cok ? (uint32_t)(px0 - HM) * pstep + 4u * (uint32_t)c : kOOB;
  const float* img = p.dy + (int64_t)n * p.H * p.W * p.dy_ps;
  auto load_row = [&](int oy, float* dst) {
    const __amdgpu_buffer_rsrc_t dr = make_rsrc(img + (int64_t)oy * p.W * p.dy_ps, rbytes);
#pragma unroll
    for (int i = 0; i < NV; ++i) dst[i] = load1(dr, loff + (uint32_t)i * pstep);
  };
  Adj3Src<0> a0;
  Adj3Src<1> a1;
  Adj3Src<2> a2;
  a0.cur = (ys + 1) >> 1;
  a1.cur = (ys + 2) >> 2;
  a2.cur = (ys + 4) >> 3;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a0.lo[j] = a0.hi[j] = 0.f;
    if (j < 4) a1.lo[j] = a1.hi[j] = 0.f;
    if (j < 2) a2.lo[j] = a2.hi[j] = 0.f;
  }
  float v[NV], nv[NV];
  load_row(ys, v);
  for (int oy = ys; oy < ye; ++oy) {
    if (oy + 1 < ye) load_row(oy + 1, nv);
    adj3_row<0, HM>(a0, v, oy, p, n, b0, b1, px0, c, cok);
    if constexpr (NUP > 1) adj3_row<1, HM>(a1, v, oy, p, n, b0, b1, px0, c, cok);
    if constexpr (NUP > 2) adj3_row<2, HM>(a2, v, oy, p, n, b0, b1, px0, c, cok);
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = nv[i];
  }
  adj3_store<0>(a0, p, n, a0.cur - 1, b0, b1, px0, c, cok);
  if constexpr (NUP > 1) adj3_store<1>(a1, p, n, a1.cur - 1, b0, b1, px0, c, cok);
  if constexpr (NUP > 2) adj3_store<2>(a2, p, n, a2.cur - 1, b0, b1, px0, c, cok);
}

// The one-pass adjoint applies: exact 2^(s+1) ratios, 64-pixel chunks, rows addressable
// with 32-bit buffer offsets.
static bool adj_one_pass(const vae2_act* dyd, int n, const vae2_act* dxds) {
  if (!g_adj_fused || n < 1 || dyd->w % kUsXB != 0 || dyd->w * dyd->ps * 4 >= (int64_t)kOOB)
    return false;
  for (int s = 0; s < n; ++s)
    if (!act_ok(&dxds[s]) || dyd->w != dxds[s].w << (s + 1) || dyd->h != dxds[s].h << (s + 1))
      return false;
  return true;
}

// The fuse layers' power-of-two adjoints (resample.hip, vae2_upsample_bilinear_bwd_pow2)
// through the one-pass kernel when its shape rules hold (targets of exactly 2 / 4 / 8, in
// that order; 64-pixel chunks); -1 when they do not (the caller takes its two-pass path).
int adj3_fuse_launch(const float* dy, const vae2_act* dyd, int n, float* const* dxs,
                     const vae2_act* dxds, const float* betas, hipStream_t st) {
  if (!g_adj_fused || !g_fuse_adj3 || n < 1 || n > 3 || !adj_one_pass(dyd, n, dxds)) return -1;
  for (int s = 0; s < n; ++s)
    if (!dxs[s] || dxds[s].n != dyd->n || dxds[s].c != dyd->c) return -1;
  UpAdj p{};
  p.dy = dy; p.dy_ps = (int)dyd->ps; p.H = (int)dyd->h; p.W = (int)dyd->w; p.C = (int)dyd->c;
  for (int s = 0; s < n; ++s) {
    p.dx[s] = dxs[s]; p.zh[s] = (int)dxds[s].h; p.zw[s] = (int)dxds[s].w;
    p.dx_ps[s] = (int)dxds[s].ps;
    p.beta[s] = betas ? betas[s] : 0.f;
  }
  p.nxb = (int)ceil_div(dyd->w, kUsXB);
  const int br = dyd->h < g_adj_band ? (int)dyd->h : g_adj_band;
  const int nband = (int)ceil_div(dyd->h, br);
  const dim3 grid((unsigned)(dyd->n * nband * p.nxb * ceil_div(dyd->c, 64)));
  switch (n) {
    case 1: VAE2_LAUNCH(up_adj3_kernel<1>, grid, dim3(256), 0, st, p, br, nband); break;
    case 2: VAE2_LAUNCH(up_adj3_kernel<2>, grid, dim3(256), 0, st, p, br, nband); break;
    default: VAE2_LAUNCH(up_adj3_kernel<3>, grid, dim3(256), 0, st, p, br, nband); break;
  }
  return 0;
}

// Pixels per block of the backward passes (>= 64 each): the reduce pass with <= 2048
// blocks (a block holds only 3 pixel rows of 68 channel quads, so 1024 blocks left one
// wave per SIMD: 134 -> 122 us per head), the apply pass with <= 1024 (measured better).
static int64_t head_ppb(int64_t P, int64_t blocks = 2048) {
  int64_t ppb = ceil_div(P, blocks);
  ppb = ppb < 64 ? 64 : ppb;
  return ppb > kHeadMaxPpb ? kHeadMaxPpb : ppb;  // the block's dout rows are staged in LDS
}

static bool head_args_ok(const float* y, const vae2_act* yd, int cout2) {
  return y && act_ok(yd) && ((uintptr_t)y % 16 == 0) && (yd->c + 3) / 4 <= 256 &&
         cout2 >= 1 && cout2 <= kHeadMaxOut;
}

#define HEAD_DISPATCH(CO_, KERNEL, ...)                                   \
  switch (CO_) {                                                          \
    case 1: VAE2_LAUNCH((KERNEL<1>), __VA_ARGS__); break;          \
    case 2: VAE2_LAUNCH((KERNEL<2>), __VA_ARGS__); break;          \
    case 3: VAE2_LAUNCH((KERNEL<3>), __VA_ARGS__); break;          \
    default: VAE2_LAUNCH((KERNEL<4>), __VA_ARGS__); break;         \
  }
// with U pixels in flight per thread (2 or 4)
#define HEAD_DISPATCH_U(CO_, U_, KERNEL, ...)                                  \
  if ((U_) == 4) {                                                             \
    switch (CO_) {                                                             \
      case 1: VAE2_LAUNCH((KERNEL<1, 4>), __VA_ARGS__); break;                 \
      case 2: VAE2_LAUNCH((KERNEL<2, 4>), __VA_ARGS__); break;                 \
      case 3: VAE2_LAUNCH((KERNEL<3, 4>), __VA_ARGS__); break;                 \
      default: VAE2_LAUNCH((KERNEL<4, 4>), __VA_ARGS__); break;                \
    }                                                                          \
  } else {                                                                     \
    HEAD_DISPATCH(CO_, KERNEL, __VA_ARGS__)                                    \
  }

}  // namespace vae2

using namespace vae2;

extern "C" {

int vae2_head_out_fwd(const float* y, const vae2_act* yd, const float* save, const float* w2,
                      const float* b2, int cout2, float* out, const vae2_act* outd,
                      void* stream) {
  const char* fn = "vae2_head_out_fwd";
  VAE2_REQUIRE(head_args_ok(y, yd, cout2) && save && w2 && out && act_ok(outd), fn,
               "bad arguments (y must be 16-byte aligned NHWC with ps % 4 == 0, cout2 <= 4)");
  VAE2_REQUIRE(outd->n == yd->n && outd->h == yd->h && outd->w == yd->w && outd->c >= cout2,
               fn, "output shape mismatch");
  const int c4 = (int)((yd->c + 3) / 4);
  const size_t shm = (size_t)(2 + cout2) * c4 * 16;
  const int64_t P = act_pixels(yd);
  const unsigned grid = (unsigned)(ceil_div(P, 16) < 8192 ? ceil_div(P, 16) : 8192);
  HEAD_DISPATCH(cout2, head_out_fwd_kernel, dim3(grid), dim3(256), shm, as_stream(stream), y,
                to_act(yd), save, w2, b2, out, to_act(outd));
  return check_launch(fn);
}

int64_t vae2_head_out_bwd_ws_size(const vae2_act* yd, int cout2) {
  if (!act_ok(yd)) return 0;
  const int64_t P = act_pixels(yd);
  const int64_t blocks = ceil_div(P, head_ppb(P));
  const int64_t NC = 2 * yd->c + cout2 * yd->c + cout2;
  return blocks * NC;
}

int vae2_head_out_bwd_reduce(const float* y, const vae2_act* yd, const float* save,
                             const float* w2, int cout2, const float* dout,
                             const vae2_act* doutd, double* sums, float* dgamma, float* dbeta,
                             float* dw2, float* db2, float* ws, int64_t ws_size, void* stream) {
  const char* fn = "vae2_head_out_bwd_reduce";
  VAE2_REQUIRE(head_args_ok(y, yd, cout2) && save && w2 && dout && sums && ws &&
                   act_ok(doutd), fn, "bad arguments");
  VAE2_REQUIRE(doutd->n == yd->n && doutd->h == yd->h && doutd->w == yd->w &&
                   doutd->c >= cout2, fn, "dout shape mismatch");
  VAE2_REQUIRE(ws_size >= vae2_head_out_bwd_ws_size(yd, cout2), fn, "workspace too small");
  const int C = (int)yd->c, c4 = (C + 3) / 4, rows = 256 / c4;
  const int NC = 2 * C + cout2 * C + cout2;
  const int64_t P = act_pixels(yd), ppb = head_ppb(P);
  const unsigned blocks = (unsigned)ceil_div(P, ppb);
  const size_t shm = ((size_t)rows * NC + (size_t)ppb * cout2) * sizeof(float);
  VAE2_REQUIRE(shm <= 64 * 1024, fn, "too many channels for the LDS reduction");
  HEAD_DISPATCH_U(cout2, g_head_red_u, head_out_bwd_reduce_kernel, dim3(blocks), dim3(256), shm,
                as_stream(stream), y, to_act(yd), save, w2, dout, to_act(doutd), ppb, rows, ws);
  int rc = check_launch(fn);
  if (rc) return rc;
  VAE2_LAUNCH(head_bwd_colsum_kernel, dim3((unsigned)ceil_div(NC, 64)), dim3(1024), 0,
                     as_stream(stream), (const float*)ws, (int)blocks, C, cout2, sums, dgamma,
                     dbeta, dw2, db2);
  return check_launch(fn);
}

int vae2_head_out_bwd_apply(const float* y, const vae2_act* yd, const float* save,
                            const float* gamma, const float* w2, int cout2, const float* dout,
                            const vae2_act* doutd, const double* sums, double count, float* dy,
                            const vae2_act* dyd, float* dbias, float* ws, int64_t ws_size,
                            void* stream) {
  const char* fn = "vae2_head_out_bwd_apply";
  VAE2_REQUIRE(head_args_ok(y, yd, cout2) && save && w2 && dout && sums && dy && ws &&
                   act_ok(doutd) && act_ok(dyd) && count > 0, fn, "bad arguments");
  VAE2_REQUIRE(doutd->n == yd->n && doutd->h == yd->h && doutd->w == yd->w &&
                   doutd->c >= cout2, fn, "dout shape mismatch");
  VAE2_REQUIRE(dyd->n == yd->n && dyd->h == yd->h && dyd->w == yd->w && dyd->c == yd->c &&
                   ((uintptr_t)dy % 16 == 0) && dyd->ps % 4 == 0, fn, "dy shape mismatch");
  VAE2_REQUIRE(ws_size >= vae2_head_out_bwd_ws_size(yd, cout2), fn, "workspace too small");
  const int C = (int)yd->c, c4 = (C + 3) / 4, rows = 256 / c4;
  const int64_t P = act_pixels(yd), ppb = head_ppb(P, 1024);
  const unsigned blocks = (unsigned)ceil_div(P, ppb);
  const size_t shm = ((size_t)rows * C + (size_t)ppb * cout2) * sizeof(float);
  HEAD_DISPATCH_U(cout2, g_head_app_u, head_out_bwd_apply_kernel, dim3(blocks), dim3(256), shm,
                as_stream(stream), y, to_act(yd), save, gamma, w2, dout, to_act(doutd), sums,
                count, ppb, rows, dy, to_act(dyd), ws);
  int rc = check_launch(fn);
  if (rc) return rc;
  if (dbias) return bias_grad_from_partials(ws, blocks, C, dbias, 1, stream);
  return 0;
}

int64_t vae2_conv1x1_upsum_stats_rows(const vae2_act* yd) {
  if (!act_ok(yd)) return 0;
  return yd->n * ceil_div(yd->h, kUsRows) * ceil_div(yd->w, kUsXB);
}

int vae2_conv1x1_upsum_fwd(const float* x, const vae2_act* xd, const float* wp,
                           const float* bias, int nup, const float* const* ups,
                           const vae2_act* upds, float* y, const vae2_act* yd, float* stats,
                           void* stream) {
  const char* fn = "vae2_conv1x1_upsum_fwd";
  VAE2_REQUIRE(x && wp && y && act_ok(xd) && act_ok(yd), fn, "bad arguments");
  VAE2_REQUIRE(xd->n == yd->n && xd->h == yd->h && xd->w == yd->w, fn, "x / y shape mismatch");
  VAE2_REQUIRE(xd->c <= kUsMaxCin, fn, "Cin0 > 32");
  VAE2_REQUIRE(nup >= 0 && nup <= 3 && (nup == 0 || (ups && upds)), fn, "bad up-sum terms");
  UpSum p{};
  p.x = x; p.x_ps = (int)xd->ps; p.cin = (int)xd->c; p.cin4 = ((int)xd->c + 3) / 4 * 4;
  p.H = (int)yd->h; p.W = (int)yd->w;
  p.wp = wp; p.bias = bias;
  const int64_t P = act_pixels(yd);
  const int64_t ncb = ceil_div(yd->c, kUsCB);
  const int64_t x_bytes = act_pixels(xd) * xd->ps * 4;
  const int64_t y_bytes = ncb * P * 64 * 4;
  VAE2_REQUIRE(x_bytes < (1ll << 31) && y_bytes < (1ll << 31), fn,
               "tensor too large for 32-bit offsets");
  p.x_bytes = (uint32_t)x_bytes;
  p.wp_bytes = (uint32_t)(ncb * kUsCB * p.cin4 * 4);
  int vtot = 0;
  for (int s = 0; s < nup; ++s) {
    const vae2_act* u = &upds[s];
    VAE2_REQUIRE(ups[s] && act_ok(u) && u->n == yd->n && u->c >= yd->c && u->h <= yd->h &&
                     u->w <= yd->w, fn, "up-sum term shape mismatch");
    const int64_t zb = act_pixels(u) * u->ps * 4;
    VAE2_REQUIRE(zb < (1ll << 31), fn, "up-sum term too large for 32-bit offsets");
    p.z[s] = ups[s]; p.zh[s] = (int)u->h; p.zw[s] = (int)u->w; p.zps[s] = (int)u->ps;
    p.z_bytes[s] = (uint32_t)zb;
    p.sh[s] = (float)u->h / (float)yd->h;
    p.sw[s] = (float)u->w / (float)yd->w;
    p.vcols[s] = (int)ceilf(p.sw[s] * kUsXB) + 3;
    VAE2_REQUIRE(p.vcols[s] <= 48, fn, "source wider than half the output (upsampling only)");
    vtot += p.vcols[s] * us_vs(s);
  }
  p.y = y; p.y_bytes = (uint32_t)y_bytes; p.C = (int)yd->c;
  p.stats = stats;
  p.nxb = (int)ceil_div(yd->w, kUsXB);
  p.nrb = (int)ceil_div(yd->h, kUsRows);
  p.rows = (int)vae2_conv1x1_upsum_stats_rows(yd);
  const int nu = nup > 0 ? nup : 1;
  const size_t shm = ((size_t)4 * nu * kUsXB + (size_t)(vtot > 0 ? vtot : 1)) * sizeof(float);
  dim3 grid((unsigned)(yd->n * p.nrb * p.nxb * ncb));
  hipStream_t st = as_stream(stream);
  bool one = g_upsum_one && yd->w % kUsXB == 0 && p.cin4 <= 20;
  for (int s = 0; s < nup; ++s)
    one = one && yd->h == (int64_t)p.zh[s] << (s + 1) && yd->w == (int64_t)p.zw[s] << (s + 1);
  if (one) {
#define US2_LAUNCH(N)                                                                   \
  switch (p.cin4 / 4) {                                                                 \
    case 1: VAE2_LAUNCH((upsum2_kernel<N, 1>), grid, dim3(256), 0, st, p); break;       \
    case 2: VAE2_LAUNCH((upsum2_kernel<N, 2>), grid, dim3(256), 0, st, p); break;       \
    case 3: VAE2_LAUNCH((upsum2_kernel<N, 3>), grid, dim3(256), 0, st, p); break;       \
    case 4: VAE2_LAUNCH((upsum2_kernel<N, 4>), grid, dim3(256), 0, st, p); break;       \
    default: VAE2_LAUNCH((upsum2_kernel<N, 5>), grid, dim3(256), 0, st, p); break;      \
  }
    switch (nup) {
      case 0: US2_LAUNCH(0) break;
      case 1: US2_LAUNCH(1) break;
      case 2: US2_LAUNCH(2) break;
      default: US2_LAUNCH(3) break;
    }
#undef US2_LAUNCH
    return check_launch(fn);
  }
  bool tight = g_upsum_tight != 0;
  for (int s = 0; s < nup; ++s) tight = tight && p.vcols[s] <= 4 * us_vu(s, true);
  const bool kq5 = p.cin4 <= 20;
#define US_LAUNCH(N)                                                                    \
  if (tight && kq5) VAE2_LAUNCH((upsum_kernel<N, true, 5>), grid, dim3(256), shm, st, p); \
  else if (tight) VAE2_LAUNCH((upsum_kernel<N, true, 8>), grid, dim3(256), shm, st, p); \
  else VAE2_LAUNCH((upsum_kernel<N, false, 8>), grid, dim3(256), shm, st, p);
  switch (nup) {
    case 0: US_LAUNCH(0) break;
    case 1: US_LAUNCH(1) break;
    case 2: US_LAUNCH(2) break;
    default: US_LAUNCH(3) break;
  }
#undef US_LAUNCH
  return check_launch(fn);
}

int64_t vae2_upsample_bilinear_bwd_multi_ws_size(const vae2_act* dyd, int n,
                                                 const vae2_act* dxds) {
  if (!act_ok(dyd) || n < 0 || n > 3 || (n && !dxds)) return 0;
  if (adj_one_pass(dyd, n, dxds)) return 1;  // no hb intermediate
  int64_t t = 0;
  for (int s = 0; s < n; ++s) t += dyd->n * dyd->h * dxds[s].w * dyd->c;
  return t > 0 ? t : 1;
}

int vae2_heads_set_algo(int algo) {
  const int prev = (g_adj_stream ? 0 : 1) | (g_upsum_tight ? 0 : 2) | (g_adj_fused ? 0 : 4) |
                   (g_upsum_one ? 0 : 8) | (g_head_red_u == 4 ? 16 : 0) |
                   (g_head_app_u == 4 ? 32 : 0) | (g_fuse_adj3 ? 64 : 0) |
                   (g_relu_dual_q ? 0 : 128) | (g_adj_band == 32 ? 0 : g_adj_band << 8);
  g_adj_stream = (algo & 1) ? 0 : 1;
  g_upsum_tight = (algo & 2) ? 0 : 1;
  g_adj_fused = (algo & 4) ? 0 : 1;
  g_upsum_one = (algo & 8) ? 0 : 1;
  g_head_red_u = (algo & 16) ? 4 : 2;
  g_head_app_u = (algo & 32) ? 4 : 2;
  g_fuse_adj3 = (algo & 64) ? 1 : 0;
  g_relu_dual_q = (algo & 128) ? 0 : 1;
  const int band = (algo >> 8) & 0xff;  // one-pass adjoint band rows (0: default 32)
  g_adj_band = band >= 8 && band % 8 == 0 ? band : 32;
  return prev;
}

int vae2_upsample_bilinear_bwd_multi(const float* dy, const vae2_act* dyd, int n,
                                     float* const* dxs, const vae2_act* dxds, float* ws,
                                     int64_t ws_size, void* stream) {
  const char* fn = "vae2_upsample_bilinear_bwd_multi";
  VAE2_REQUIRE(dy && act_ok(dyd) && n >= 0 && n <= 3 && (n == 0 || (dxs && dxds)) && ws, fn,
               "bad arguments");
  VAE2_REQUIRE(ws_size >= vae2_upsample_bilinear_bwd_multi_ws_size(dyd, n, dxds), fn,
               "workspace too small");
  if (n == 0) return 0;
  UpAdj p{};
  p.dy = dy; p.dy_ps = (int)dyd->ps; p.H = (int)dyd->h; p.W = (int)dyd->w; p.C = (int)dyd->c;
  float* hb = ws;
  float min_sw = 1.f;
  for (int s = 0; s < n; ++s) {
    const vae2_act* d = &dxds[s];
    VAE2_REQUIRE(dxs[s] && act_ok(d) && d->n == dyd->n && d->c == dyd->c && d->h <= dyd->h &&
                     d->w <= dyd->w, fn, "dx shape mismatch");
    p.dx[s] = dxs[s]; p.zh[s] = (int)d->h; p.zw[s] = (int)d->w; p.dx_ps[s] = (int)d->ps;
    p.sh[s] = (float)d->h / (float)dyd->h;
    p.sw[s] = (float)d->w / (float)dyd->w;
    VAE2_REQUIRE(2.f / p.sh[s] + 6.f <= 64.f, fn, "upsampling ratio too large (> 24)");
    if (p.sw[s] < min_sw) min_sw = p.sw[s];
    p.hb[s] = hb;
    hb += dyd->n * dyd->h * d->w * dyd->c;
  }
  p.nxb = (int)ceil_div(dyd->w, kUsXB);
  const unsigned cb = (unsigned)ceil_div(dyd->c, 64);
  hipStream_t st = as_stream(stream);
  bool pow2 = dyd->w % kUsXB == 0;
  for (int s = 0; s < n; ++s)
    pow2 = pow2 && dyd->w == (int64_t)p.zw[s] << (s + 1) && dyd->h == (int64_t)p.zh[s] << (s + 1);
  if (adj_one_pass(dyd, n, dxds)) {
    const int br = dyd->h < g_adj_band ? (int)dyd->h : g_adj_band;
    const int nband = (int)ceil_div(dyd->h, br);
    const dim3 grid((unsigned)(dyd->n * nband * p.nxb * cb));
    switch (n) {
      case 1: VAE2_LAUNCH(up_adj3_kernel<1>, grid, dim3(256), 0, st, p, br, nband); break;
      case 2: VAE2_LAUNCH(up_adj3_kernel<2>, grid, dim3(256), 0, st, p, br, nband); break;
      default: VAE2_LAUNCH(up_adj3_kernel<3>, grid, dim3(256), 0, st, p, br, nband); break;
    }
    return check_launch(fn);
  }
  if (pow2) {
    const dim3 grid((unsigned)(dyd->n * dyd->h * p.nxb * cb));
    switch (n) {
      case 1: VAE2_LAUNCH(up_adj2_h_kernel<1>, grid, dim3(256), 0, st, p); break;
      case 2: VAE2_LAUNCH(up_adj2_h_kernel<2>, grid, dim3(256), 0, st, p); break;
      default: VAE2_LAUNCH(up_adj2_h_kernel<3>, grid, dim3(256), 0, st, p); break;
    }
    int rc = check_launch(fn);
    if (rc) return rc;
    for (int s = 0; s < n; ++s) {
      const int64_t rs = (int64_t)p.zw[s] * p.C;
      if (rs % 4 == 0 && g_adj_stream) {
        const int64_t nq = rs / 4;
        const dim3 gv((unsigned)(dyd->n * p.zh[s]), (unsigned)ceil_div(nq, 512));
        const FastDiv cdiv((uint32_t)p.C);
        switch (s) {
          case 0: VAE2_LAUNCH(up_adj2_vs_kernel<0>, gv, dim3(256), 0, st, p, cdiv); break;
          case 1: VAE2_LAUNCH(up_adj2_vs_kernel<1>, gv, dim3(256), 0, st, p, cdiv); break;
          default: VAE2_LAUNCH(up_adj2_vs_kernel<2>, gv, dim3(256), 0, st, p, cdiv); break;
        }
      } else {
        const dim3 gv((unsigned)(dyd->n * p.zh[s]), cb);
        switch (s) {
          case 0: VAE2_LAUNCH(up_adj2_v_kernel<0>, gv, dim3(256), 0, st, p); break;
          case 1: VAE2_LAUNCH(up_adj2_v_kernel<1>, gv, dim3(256), 0, st, p); break;
          default: VAE2_LAUNCH(up_adj2_v_kernel<2>, gv, dim3(256), 0, st, p); break;
        }
      }
      rc = check_launch(fn);
      if (rc) return rc;
    }
    return 0;
  }
  // halo: the owned columns' windows reach at most 1/sw + 3 pixels past the chunk
  p.halo = (int)ceilf(1.f / min_sw) + 4;
  const int span = kUsXB + 2 * p.halo;
  const size_t shm = (size_t)(4 * n + 64) * span * sizeof(float);
  VAE2_REQUIRE(shm <= 64 * 1024, fn, "upsampling ratio too large for the LDS tile");
  dim3 grid((unsigned)(dyd->n * dyd->h * p.nxb * cb));
  switch (n) {
    case 1: VAE2_LAUNCH(up_adj_h_kernel<1>, grid, dim3(256), shm, st, p); break;
    case 2: VAE2_LAUNCH(up_adj_h_kernel<2>, grid, dim3(256), shm, st, p); break;
    default: VAE2_LAUNCH(up_adj_h_kernel<3>, grid, dim3(256), shm, st, p); break;
  }
  int rc = check_launch(fn);
  if (rc) return rc;
  for (int s = 0; s < n; ++s) {
    VAE2_LAUNCH(up_adj_v_kernel, dim3((unsigned)(dyd->n * p.zh[s]), cb), dim3(256), 0, st,
                       p, s);
    rc = check_launch(fn);
    if (rc) return rc;
  }
  return 0;
}

}  // extern "C"
