// Convolutions of the HRNet stacks as implicit GEMMs on the fp32 matrix cores
// (v_mfma_f32_16x16x4_f32: exact fp32 FMA chains, 64 FLOP/clk/SIMD on gfx950).
//
//   forward     Y[m][n]  = sum_k A[m][k] * B[k][n]
//               m = output pixel, n = Cout, k = (tap, Cin); A = im2col(X) gathered
//               on the fly from NHWC, B = W[Cout][Cin][kh][kw] read in place.
//   bwd data    same kernel: m = input pixel (one stride-parity class per launch),
//               n = Cin, k = (valid tap, Cout), A = dY gathered, B = W^T.
//   bwd weight  dW[co][(tap,ci)] = sum_p dY[p][co] * X[src(p,tap)][ci], split over
//               pixels (split-K) into fp32 slabs, then a fixed-order reduction
//               into the [Cout][Cin][kh][kw] gradient (deterministic).
//
// Replaces nn.Conv2d forward/backward for every conv of enc_hrnet.py (see
// include/vae2_hip.h for the call sites).
//
// K ordering trick: within each 16-deep K chunk, lane group g = lane>>4 owns
// k = 4g..4g+3, and MFMA k-step s uses k = 4g+s for both operands.  The A and B
// fragments of all four k-steps then come from ONE 16-byte LDS read per lane
// (layout [g][row][4], conflict-free for ds_read_b128) — a permutation of the
// reduction order that the sum does not see.
#include "common.h"

namespace vae2 {

typedef float f4 __attribute__((ext_vector_type(4)));

struct IGemm {
  // A operand: activation gathered from NHWC
  const float* a;
  int64_t a_ps;
  int a_c, a_h, a_w;
  // iteration grid: M = g_n * g_h * g_w rows
  int g_n, g_h, g_w;
  int a_step;  // A source row = g*a_step + d(tap)
  // taps: t = th*ntw + tw;  d = d0 + th*ds;  weight tap (kh0 + th*khs, kw0 + tw*kws)
  int nth, ntw;
  int dh0, dhs, dw0, dws;
  int kh0, khs, kw0, kws, kw_size;
  // B operand: B[n][(t, c)] = w[n*w_sn + c*w_sc + kh*kw_size + kw]
  const float* w;
  int64_t w_sn, w_sc;
  int n;
  const float* bias;
  // output: row (gi*y_step + y_offh), col (gj*y_step + y_offw)
  float* y;
  int64_t y_ps;
  int y_h, y_w, y_step, y_offh, y_offw;
  float beta;
  float* stats;  // [2][gridDim.x][n] or null
};

constexpr int BK = 16;

// ROLE only separates forward (0) and data-gradient (1) launches in profiles.
template <int TM, int TN, int ROLE>
__global__ __launch_bounds__(256) void igemm_kernel(IGemm p) {
  constexpr int BM = 64 * TM;
  constexpr int BN = 16 * TN;
  constexpr int A_F = 4 * BM * 4;  // floats per A buffer: [4 groups][BM][4]
  constexpr int B_F = 4 * BN * 4;
  __shared__ __attribute__((aligned(16))) float smem[2 * (A_F + B_F)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int64_t M = (int64_t)p.g_n * p.g_h * p.g_w;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int ntaps = p.nth * p.ntw;
  const int K = ntaps * p.a_c;
  const int nchunks = (K + BK - 1) / BK;

  // ---- per-thread gather rows (A) ----
  const int q = tid & 3;          // k quad owned by this thread in a chunk
  const int rbase = tid >> 2;     // 0..63
  int64_t a_img[TM];
  int a_i[TM], a_j[TM];
  bool a_ok[TM];
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    int64_t m = m0 + rbase + 64 * j;
    a_ok[j] = m < M;
    int64_t mm = a_ok[j] ? m : 0;
    int64_t hw = (int64_t)p.g_h * p.g_w;
    int64_t gn = mm / hw;
    int64_t rem = mm - gn * hw;
    int gi = (int)(rem / p.g_w);
    int gj = (int)(rem - (int64_t)gi * p.g_w);
    a_img[j] = gn * p.a_h;
    a_i[j] = gi * p.a_step;
    a_j[j] = gj * p.a_step;
  }
  // B rows owned by this thread
  constexpr int BROWS = (BN + 63) / 64;
  // (tap, channel) of k = chunk*16 + 4q
  int tb = 0, cb = 4 * q;
  while (cb >= p.a_c) { cb -= p.a_c; ++tb; }

  float ra[TM][4];
  float rb[BROWS][4];

  auto load_chunk = [&](int chunk_t, int chunk_c) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int t = chunk_t, c = chunk_c + e;
      while (c >= p.a_c) { c -= p.a_c; ++t; }
      bool tv = t < ntaps;
      int th = tv ? t / p.ntw : 0;
      int tw = tv ? t - th * p.ntw : 0;
      int dh = p.dh0 + th * p.dhs;
      int dw = p.dw0 + tw * p.dws;
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        int ih = a_i[j] + dh, iw = a_j[j] + dw;
        bool ok = tv && a_ok[j] && ih >= 0 && ih < p.a_h && iw >= 0 && iw < p.a_w;
        float v = 0.f;
        if (ok) v = p.a[((a_img[j] + ih) * p.a_w + iw) * p.a_ps + c];
        ra[j][e] = v;
      }
      int kh = p.kh0 + th * p.khs, kw = p.kw0 + tw * p.kws;
      int64_t toff = (int64_t)kh * p.kw_size + kw;
#pragma unroll
      for (int j = 0; j < BROWS; ++j) {
        int nr = rbase + 64 * j;
        float v = 0.f;
        if (tv && nr < BN && n0 + nr < p.n)
          v = p.w[(int64_t)(n0 + nr) * p.w_sn + (int64_t)c * p.w_sc + toff];
        rb[j][e] = v;
      }
    }
  };
  auto store_chunk = [&](int buf) {
    float* As = smem + buf * (A_F + B_F);
    float* Bs = As + A_F;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      f4 v = {ra[j][0], ra[j][1], ra[j][2], ra[j][3]};
      *reinterpret_cast<f4*>(As + (q * BM + rbase + 64 * j) * 4) = v;
    }
#pragma unroll
    for (int j = 0; j < BROWS; ++j) {
      int nr = rbase + 64 * j;
      if (nr < BN) {
        f4 v = {rb[j][0], rb[j][1], rb[j][2], rb[j][3]};
        *reinterpret_cast<f4*>(Bs + (q * BN + nr) * 4) = v;
      }
    }
  };

  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, r = lane & 15;
  const int wm0 = wave * 16 * TM;

  if (nchunks > 0) load_chunk(tb, cb);
  for (int ch = 0; ch < nchunks; ++ch) {
    const int buf = ch & 1;
    store_chunk(buf);
    __syncthreads();
    if (ch + 1 < nchunks) {
      cb += BK;
      while (cb >= p.a_c) { cb -= p.a_c; ++tb; }
      load_chunk(tb, cb);
    }
    const float* As = smem + buf * (A_F + B_F);
    const float* Bs = As + A_F;
    f4 fa[TM], fb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
      fa[i] = *reinterpret_cast<const f4*>(As + (g * BM + wm0 + i * 16 + r) * 4);
#pragma unroll
    for (int j = 0; j < TN; ++j)
      fb[j] = *reinterpret_cast<const f4*>(Bs + (g * BN + j * 16 + r) * 4);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
  }

  // ---- epilogue ----
  const int64_t hw = (int64_t)p.g_h * p.g_w;
  float csum[TN], csq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) { csum[j] = 0.f; csq[j] = 0.f; }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int64_t m = m0 + wm0 + i * 16 + g * 4 + e;
      if (m >= M) continue;
      int64_t gn = m / hw;
      int64_t rem = m - gn * hw;
      int gi = (int)(rem / p.g_w);
      int gj = (int)(rem - (int64_t)gi * p.g_w);
      int64_t oy = (int64_t)gi * p.y_step + p.y_offh;
      int64_t ox = (int64_t)gj * p.y_step + p.y_offw;
      float* yrow = p.y + ((gn * p.y_h + oy) * p.y_w + ox) * p.y_ps;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int n = n0 + j * 16 + r;
        if (n >= p.n) continue;
        float v = acc[i][j][e];
        if (p.bias) v += p.bias[n];
        if (p.beta != 0.f) v += p.beta * yrow[n];
        yrow[n] = v;
        csum[j] += v;
        csq[j] += v * v;
      }
    }
  }
  if (p.stats) {
    // reduce over the 4 row groups of the wave (lanes r, r+16, r+32, r+48)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      csum[j] += __shfl_xor(csum[j], 16, 64);
      csum[j] += __shfl_xor(csum[j], 32, 64);
      csq[j] += __shfl_xor(csq[j], 16, 64);
      csq[j] += __shfl_xor(csq[j], 32, 64);
    }
    __syncthreads();  // done with operand buffers: reuse smem
    float* red = smem;  // [4 waves][2][BN]
    if (g == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        red[(wave * 2 + 0) * BN + j * 16 + r] = csum[j];
        red[(wave * 2 + 1) * BN + j * 16 + r] = csq[j];
      }
    }
    __syncthreads();
    const int64_t rows = gridDim.x;
    for (int c = tid; c < BN; c += 256) {
      if (n0 + c >= p.n) continue;
      float s = 0.f, s2 = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        s += red[(w * 2 + 0) * BN + c];
        s2 += red[(w * 2 + 1) * BN + c];
      }
      p.stats[(int64_t)blockIdx.x * p.n + n0 + c] = s;
      p.stats[(rows + blockIdx.x) * p.n + n0 + c] = s2;
    }
  }
}

// ------------------------------------------------------------ tiling ----
struct Tile {
  int tm, tn, nblk;
};

static Tile pick_tile(int64_t M, int N) {
  Tile t;
  int tiles = (N + 15) / 16;
  if (tiles <= 9) {
    t.tn = tiles;
    t.nblk = 1;
  } else {
    t.nblk = (tiles + 7) / 8;
    t.tn = (tiles + t.nblk - 1) / t.nblk;
  }
  t.tm = (M >= 128 * 256) ? 2 : 1;
  return t;
}

template <int TM, int ROLE>
static void launch_tn(const IGemm& p, int tn, dim3 grid, hipStream_t s) {
  switch (tn) {
#define CASE(T) \
  case T: hipLaunchKernelGGL((igemm_kernel<TM, T, ROLE>), grid, dim3(256), 0, s, p); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9)
#undef CASE
  }
}

static int launch_igemm(const IGemm& p, int role, hipStream_t s, const char* fn) {
  int64_t M = (int64_t)p.g_n * p.g_h * p.g_w;
  if (M == 0) return 0;
  Tile t = pick_tile(M, p.n);
  dim3 grid((unsigned)ceil_div(M, 64 * t.tm), (unsigned)t.nblk);
  if (role == 0) {
    if (t.tm == 2) launch_tn<2, 0>(p, t.tn, grid, s);
    else launch_tn<1, 0>(p, t.tn, grid, s);
  } else {
    if (t.tm == 2) launch_tn<2, 1>(p, t.tn, grid, s);
    else launch_tn<1, 1>(p, t.tn, grid, s);
  }
  return check_launch(fn);
}

static int64_t igemm_rows(int64_t M, int N) {
  Tile t = pick_tile(M, N);
  return ceil_div(M, 64 * t.tm);
}

// ------------------------------------------------------------ wgrad ----
struct WGrad {
  const float* x;  // B operand source (NHWC)
  int64_t x_ps;
  int cin, x_h, x_w;
  const float* dy;  // A operand source (NHWC)
  int64_t dy_ps;
  int cout, o_n, o_h, o_w;
  int k, stride, pad;
  int64_t P;          // o_n*o_h*o_w
  int64_t px_split;   // pixels per split (multiple of 16)
  float* part;        // [split][cout][ncol], ncol = k*k*cin
};

// Block: 4 waves along the (tap, cin) columns; wave tile 16*TM rows (cout) x 16*TN cols.
template <int TM, int TN>
__global__ __launch_bounds__(256) void wgrad_kernel(WGrad p) {
  constexpr int BM = 16 * TM;       // cout rows per block
  constexpr int BN = 64 * TN;       // (tap, cin) columns per block
  constexpr int A_F = 4 * BM * 4;   // [g][BM][4]
  constexpr int B_F = 4 * BN * 4;
  __shared__ __attribute__((aligned(16))) float smem[2 * (A_F + B_F)];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ncol = p.k * p.k * p.cin;
  const int co0 = blockIdx.y * BM;
  const int col0 = blockIdx.x * BN;
  const int64_t pbeg = (int64_t)blockIdx.z * p.px_split;
  int64_t pend = pbeg + p.px_split;
  if (pend > p.P) pend = p.P;
  const int nchunks = (int)((pend - pbeg + BK - 1) / BK);

  // Loading: A' tile BM x 16 pixels; B' tile BN x 16 pixels.
  // thread -> (quad q of pixels, row) : q = tid & 3, rows tid>>2 (+64j)
  const int q = tid & 3, rbase = tid >> 2;
  constexpr int AROWS = (BM + 63) / 64;
  constexpr int BROWS = BN / 64;  // == TN
  // B' column decomposition (tap, ci) per owned row
  int b_kh[BROWS], b_kw[BROWS], b_ci[BROWS];
  bool b_ok[BROWS];
#pragma unroll
  for (int j = 0; j < BROWS; ++j) {
    int col = col0 + rbase + 64 * j;
    b_ok[j] = col < ncol;
    int cc = b_ok[j] ? col : 0;
    int t = cc / p.cin;
    b_ci[j] = cc - t * p.cin;
    b_kh[j] = t / p.k;
    b_kw[j] = t - b_kh[j] * p.k;
  }
  float ra[AROWS][4], rb[BROWS][4];
  const int64_t ohw = (int64_t)p.o_h * p.o_w;

  auto load_chunk = [&](int64_t pc) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int64_t pix = pc + 4 * q + e;
      bool pv = pix < pend;
      int64_t pp = pv ? pix : 0;
      int64_t n = pp / ohw;
      int64_t rem = pp - n * ohw;
      int oh = (int)(rem / p.o_w);
      int ow = (int)(rem - (int64_t)oh * p.o_w);
      const float* dyrow = p.dy + pp * p.dy_ps;
#pragma unroll
      for (int j = 0; j < AROWS; ++j) {
        int co = co0 + rbase + 64 * j;
        float v = 0.f;
        if (pv && rbase + 64 * j < BM && co < p.cout) v = dyrow[co];
        ra[j][e] = v;
      }
#pragma unroll
      for (int j = 0; j < BROWS; ++j) {
        int ih = oh * p.stride - p.pad + b_kh[j];
        int iw = ow * p.stride - p.pad + b_kw[j];
        float v = 0.f;
        if (pv && b_ok[j] && ih >= 0 && ih < p.x_h && iw >= 0 && iw < p.x_w)
          v = p.x[((n * p.x_h + ih) * p.x_w + iw) * p.x_ps + b_ci[j]];
        rb[j][e] = v;
      }
    }
  };
  auto store_chunk = [&](int buf) {
    float* As = smem + buf * (A_F + B_F);
    float* Bs = As + A_F;
#pragma unroll
    for (int j = 0; j < AROWS; ++j) {
      int rr = rbase + 64 * j;
      if (rr < BM) {
        f4 v = {ra[j][0], ra[j][1], ra[j][2], ra[j][3]};
        *reinterpret_cast<f4*>(As + (q * BM + rr) * 4) = v;
      }
    }
#pragma unroll
    for (int j = 0; j < BROWS; ++j) {
      f4 v = {rb[j][0], rb[j][1], rb[j][2], rb[j][3]};
      *reinterpret_cast<f4*>(Bs + (q * BN + rbase + 64 * j) * 4) = v;
    }
  };

  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, r = lane & 15;
  const int wn0 = wave * 16 * TN;

  if (nchunks > 0) load_chunk(pbeg);
  for (int ch = 0; ch < nchunks; ++ch) {
    const int buf = ch & 1;
    store_chunk(buf);
    __syncthreads();
    if (ch + 1 < nchunks) load_chunk(pbeg + (int64_t)(ch + 1) * BK);
    const float* As = smem + buf * (A_F + B_F);
    const float* Bs = As + A_F;
    f4 fa[TM], fb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
      fa[i] = *reinterpret_cast<const f4*>(As + (g * BM + i * 16 + r) * 4);
#pragma unroll
    for (int j = 0; j < TN; ++j)
      fb[j] = *reinterpret_cast<const f4*>(Bs + (g * BN + wn0 + j * 16 + r) * 4);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
  }

  float* out = p.part + (int64_t)blockIdx.z * p.cout * ncol;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int co = co0 + i * 16 + g * 4 + e;
      if (co >= p.cout) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int col = col0 + wn0 + j * 16 + r;
        if (col < ncol) out[(int64_t)co * ncol + col] = acc[i][j][e];
      }
    }
}

// dw[co][ci][kh][kw] (+)= sum_s part[s][co][(kh*k+kw)*cin + ci]
__global__ void wgrad_reduce_kernel(const float* part, int64_t splits, int cout,
                                    int cin, int k, float* dw, int accumulate) {
  const int ncol = k * k * cin;
  const int64_t total = (int64_t)cout * ncol;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int co = (int)(idx / ncol);
    int col = (int)(idx - (int64_t)co * ncol);
    float s = 0.f;
    for (int64_t sp = 0; sp < splits; ++sp) s += part[sp * total + idx];
    int t = col / cin;
    int ci = col - t * cin;
    int64_t o = ((int64_t)co * cin + ci) * (k * k) + t;
    dw[o] = accumulate ? dw[o] + s : s;
  }
}

struct WTile {
  int tm, tn;
  int64_t splits, px_split;
  int gx, gy;
};

static WTile pick_wtile(int64_t P, int cout, int ncol) {
  WTile t;
  int mt = (cout + 15) / 16;
  t.tm = mt <= 4 ? mt : 4;
  int ct = (ncol + 63) / 64;  // 64-column units
  t.tn = ct <= 2 ? ct : 2;
  t.gy = (int)ceil_div(cout, 16 * t.tm);
  t.gx = (int)ceil_div(ncol, 64 * t.tn);
  int64_t tiles = (int64_t)t.gx * t.gy;
  // aim for ~2048 workgroups, at least 256 pixels (16 chunks) per split
  int64_t want = ceil_div(2048, tiles);
  int64_t maxs = ceil_div(P, 256);
  int64_t s = want < maxs ? want : maxs;
  if (s < 1) s = 1;
  t.px_split = ceil_div(ceil_div(P, s), BK) * BK;
  t.splits = ceil_div(P, t.px_split);
  return t;
}

template <int TM>
static void launch_wgrad_tn(const WGrad& p, int tn, dim3 grid, hipStream_t s) {
  if (tn == 1)
    hipLaunchKernelGGL((wgrad_kernel<TM, 1>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((wgrad_kernel<TM, 2>), grid, dim3(256), 0, s, p);
}

// ------------------------------------------------------------- checks ----
static bool conv_shapes_ok(const vae2_act* xd, const vae2_act* yd, int k,
                           int stride, int pad) {
  if (!act_ok(xd) || !act_ok(yd)) return false;
  if (xd->n != yd->n) return false;
  if (k < 1 || stride < 1 || pad < 0) return false;
  int64_t oh = (xd->h + 2 * pad - k) / stride + 1;
  int64_t ow = (xd->w + 2 * pad - k) / stride + 1;
  return oh == yd->h && ow == yd->w;
}

}  // namespace vae2

using namespace vae2;

extern "C" {

int64_t vae2_conv2d_fwd_stats_rows(const vae2_act* yd, int64_t cout) {
  return igemm_rows(act_pixels(yd), (int)cout);
}

int vae2_conv2d_fwd_kernel_name(const vae2_act* yd, int64_t cout, char* buf, int64_t len) {
  if (!yd || !buf || len <= 0) return -22;
  Tile t = pick_tile(act_pixels(yd), (int)cout);
  snprintf(buf, (size_t)len, "igemm_kernel<%d, %d, 0>", t.tm, t.tn);
  return 0;
}

int vae2_conv2d_fwd(const float* x, const vae2_act* xd, const float* w,
                    const float* bias, float* y, const vae2_act* yd, int k,
                    int stride, int pad, float beta, float* stats,
                    void* stream) {
  const char* fn = "vae2_conv2d_fwd";
  VAE2_REQUIRE(x && w && y, fn, "null pointer");
  VAE2_REQUIRE(conv_shapes_ok(xd, yd, k, stride, pad), fn, "inconsistent conv shapes");
  IGemm p{};
  p.a = x; p.a_ps = xd->ps; p.a_c = (int)xd->c; p.a_h = (int)xd->h; p.a_w = (int)xd->w;
  p.g_n = (int)yd->n; p.g_h = (int)yd->h; p.g_w = (int)yd->w;
  p.a_step = stride;
  p.nth = k; p.ntw = k;
  p.dh0 = -pad; p.dhs = 1; p.dw0 = -pad; p.dws = 1;
  p.kh0 = 0; p.khs = 1; p.kw0 = 0; p.kws = 1; p.kw_size = k;
  p.w = w; p.w_sn = xd->c * k * k; p.w_sc = (int64_t)k * k; p.n = (int)yd->c;
  p.bias = bias;
  p.y = y; p.y_ps = yd->ps; p.y_h = (int)yd->h; p.y_w = (int)yd->w;
  p.y_step = 1; p.y_offh = 0; p.y_offw = 0;
  p.beta = beta;
  p.stats = stats;
  return launch_igemm(p, 0, as_stream(stream), fn);
}

int vae2_conv2d_bwd_data(const float* dy, const vae2_act* dyd, const float* w,
                         float* dx, const vae2_act* dxd, int k, int stride,
                         int pad, float beta, void* stream) {
  const char* fn = "vae2_conv2d_bwd_data";
  VAE2_REQUIRE(dy && w && dx, fn, "null pointer");
  VAE2_REQUIRE(conv_shapes_ok(dxd, dyd, k, stride, pad), fn, "inconsistent conv shapes");
  // One launch per (ph, pw) stride-parity class of the input pixels.
  // Input row ih = stride*i + ph receives from output row oh = (ih + pad - kh)/stride
  // for every kh with (ph + pad - kh) % stride == 0.
  for (int ph = 0; ph < stride; ++ph) {
    for (int pw = 0; pw < stride; ++pw) {
      int gh = (int)((dxd->h - ph + stride - 1) / stride);
      int gw = (int)((dxd->w - pw + stride - 1) / stride);
      if (gh <= 0 || gw <= 0) continue;
      // valid kh: kh0, kh0+stride, ... < k, with (ph + pad - kh0) % stride == 0
      int kh0 = ((ph + pad) % stride + stride) % stride;
      int kw0 = ((pw + pad) % stride + stride) % stride;
      int nth = kh0 < k ? (k - 1 - kh0) / stride + 1 : 0;
      int ntw = kw0 < k ? (k - 1 - kw0) / stride + 1 : 0;
      IGemm p{};
      p.a = dy; p.a_ps = dyd->ps; p.a_c = (int)dyd->c; p.a_h = (int)dyd->h; p.a_w = (int)dyd->w;
      p.g_n = (int)dxd->n; p.g_h = gh; p.g_w = gw;
      p.a_step = 1;
      p.nth = nth; p.ntw = ntw;
      // oh = i + (ph + pad - kh)/stride ; kh = kh0 + th*stride -> d = d0 - th
      p.dh0 = (ph + pad - kh0) / stride; p.dhs = -1;
      p.dw0 = (pw + pad - kw0) / stride; p.dws = -1;
      p.kh0 = kh0; p.khs = stride; p.kw0 = kw0; p.kws = stride; p.kw_size = k;
      // B[n = ci][(t, c = co)] = w[co][ci][kh][kw]
      p.w = w; p.w_sn = (int64_t)k * k; p.w_sc = dxd->c * k * k; p.n = (int)dxd->c;
      p.bias = nullptr;
      p.y = dx; p.y_ps = dxd->ps; p.y_h = (int)dxd->h; p.y_w = (int)dxd->w;
      p.y_step = stride; p.y_offh = ph; p.y_offw = pw;
      p.beta = beta;
      p.stats = nullptr;
      if (nth == 0 || ntw == 0) { p.nth = 0; p.ntw = 1; }
      int rc = launch_igemm(p, 1, as_stream(stream), fn);
      if (rc) return rc;
    }
  }
  return 0;
}

int64_t vae2_conv2d_bwd_weight_ws_size(const vae2_act* xd, const vae2_act* dyd,
                                       int k) {
  if (!act_ok(xd) || !act_ok(dyd)) return 0;
  int ncol = (int)(k * k * xd->c);
  WTile t = pick_wtile(act_pixels(dyd), (int)dyd->c, ncol);
  int64_t part = t.splits * dyd->c * ncol;
  int64_t bias_part = 2 * vae2_bn_partial_rows(dyd) * dyd->c;
  int64_t bias_sums = 2 * dyd->c * 2;  // doubles as floats
  return part + bias_part + bias_sums + 4;
}

int vae2_conv2d_bwd_weight(const float* x, const vae2_act* xd, const float* dy,
                           const vae2_act* dyd, float* dw, float* dbias, int k,
                           int stride, int pad, int accumulate, float* ws,
                           int64_t ws_size, void* stream) {
  const char* fn = "vae2_conv2d_bwd_weight";
  VAE2_REQUIRE(x && dy && dw && ws, fn, "null pointer");
  VAE2_REQUIRE(conv_shapes_ok(xd, dyd, k, stride, pad), fn, "inconsistent conv shapes");
  VAE2_REQUIRE(ws_size >= vae2_conv2d_bwd_weight_ws_size(xd, dyd, k), fn, "workspace too small");
  hipStream_t s = as_stream(stream);
  int ncol = (int)(k * k * xd->c);
  WTile t = pick_wtile(act_pixels(dyd), (int)dyd->c, ncol);
  WGrad p{};
  p.x = x; p.x_ps = xd->ps; p.cin = (int)xd->c; p.x_h = (int)xd->h; p.x_w = (int)xd->w;
  p.dy = dy; p.dy_ps = dyd->ps; p.cout = (int)dyd->c;
  p.o_n = (int)dyd->n; p.o_h = (int)dyd->h; p.o_w = (int)dyd->w;
  p.k = k; p.stride = stride; p.pad = pad;
  p.P = act_pixels(dyd);
  p.px_split = t.px_split;
  p.part = ws;
  dim3 grid(t.gx, t.gy, (unsigned)t.splits);
  switch (t.tm) {
    case 1: launch_wgrad_tn<1>(p, t.tn, grid, s); break;
    case 2: launch_wgrad_tn<2>(p, t.tn, grid, s); break;
    case 3: launch_wgrad_tn<3>(p, t.tn, grid, s); break;
    default: launch_wgrad_tn<4>(p, t.tn, grid, s); break;
  }
  int rc = check_launch(fn);
  if (rc) return rc;
  int64_t total = (int64_t)dyd->c * ncol;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(ew_blocks(total)), dim3(256), 0, s,
                     (const float*)ws, t.splits, (int)dyd->c, (int)xd->c, k, dw, accumulate);
  rc = check_launch(fn);
  if (rc) return rc;
  if (dbias) {
    float* bp = ws + t.splits * dyd->c * ncol;
    rc = vae2_bn_stats(dy, dyd, bp, stream);
    if (rc) return rc;
    rc = bias_grad_from_partials(bp, vae2_bn_partial_rows(dyd), dyd->c, dbias,
                                      accumulate, stream);
    if (rc) return rc;
  }
  return 0;
}

}  // extern "C"
