// Narrow-channel 3x3 stride-1 weight gradient (the HRNet branches: 18 / 36 / 72 channels,
// enc_hrnet.py:27-30 conv3x3 inside BasicBlock, :33-62).
//
//   dW[co][ci][dh][dw] = sum_px dY[px][co] * X[px + (dh-1, dw-1)][ci]
//
// GEMM view: M = co (16*TM on MFMA + NR <= 4 on the VALU), K = output pixels, N = the 9*ci
// (tap, channel) columns.  wgrad3_kernel (conv.hip) orders the columns (tap, ci) and reads
// every B fragment (4 consecutive pixels of one column) as four unaligned LDS words.  Here
// the columns are ordered (dw, dh, ci) with every dw group padded to whole 16-column tiles:
// lane (r, g) of column tile (j, dw) holds column (dh, ci) = divmod(16 j + r, CSW) for all
// three dw, and the three B fragments are windows of ONE run of 6 consecutive halo pixels
// (4 pixels of its lane group + the 2 tap shifts) -- 6 LDS reads feed 3 * 4 * TM MFMAs.
// Both tiles stay pixel-major in LDS (the NHWC layout): the staging is 16-byte loads and
// 16-byte LDS writes, no transposition.  The A fragment (dY, 4 pixels x 16 co) is read once
// per 16-pixel chunk and reused by every column tile of the wave.
//
// Work split: a workgroup (4 waves) walks `tps` tiles of TH x 32 output pixels (split-K:
// its partial dW slab goes to part[split], summed by wgrad_reduce_kernel in a fixed
// order); the next tile's global loads are in flight (registers) while the current tile
// computes.  WPIX waves split the tile's 16-pixel chunks, the remaining factor 4 / WPIX
// splits the column groups; waves holding the same columns are summed through LDS at the
// end in a fixed order (deterministic).
#include "common.h"

namespace vae2 {

extern int g_bf16, g_wgrad_narrow;
int g_wgrad_narrow_tps = 2;  // vae2_conv2d_set_tune key 16: minimum tiles per split (1 or 2)

// (the kernel is an exported symbol, outside the anonymous namespace: the launch log
// names kernels through the dynamic symbol table)
constexpr int kTH = 4;            // output rows per tile
constexpr int kTW = 32;           // output columns per tile
constexpr int kLW = kTW + 2;      // halo columns
constexpr int kNPX = kTH * kTW;   // output pixels per tile

struct WGN {
  const float* x;
  int x_ps, cin, cin4, h, w;
  const float* dy;
  int dy_ps, cout;
  int tiles_h, tiles_w, ntiles, tps;
  int n_ci_slabs;
  FastDiv per_img_div, tiles_w_div;  // tile index -> (image, tile row, tile column)
  uint32_t x_bytes, dy_bytes;
  float* part;  // [splits][cout][9 * cin4], column = (dh * 3 + dw) * cin4 + ci
  // x is the pre-BN output of a BatchNorm(+ReLU) layer whose normalised activation is never
  // stored (LazyBN): the staging applies relu?(x * scale + shift) to in-image pixels
  const float* isave;
  int irelu;
};

// CQ: channel quads per ci slab (CSW = 4 CQ columns per (dh, dw)); TM: 16-row co tiles on
// MFMA; NR: remainder co rows on the VALU (<= 4, one staged quad); WPIX: waves splitting the
// pixels of a tile (1, 2 or 4); PF: the next tile's loads in registers during the current
// tile's MFMAs (else the resident workgroups of a CU overlap each other's staging).
// NW: waves per workgroup (4, or 8: twice the waves per SIMD for the same tiles and partial
// slabs, the extra waves splitting the pixel chunks -- set_tune key 7 = 3)
template <int CQ, int TM, int NR, int WPIX, bool PF, int NW = 4>
__global__ __launch_bounds__(64 * NW) void wgrad3n_kernel(WGN p) {
  constexpr int CSW = 4 * CQ;
  constexpr int CO = 16 * TM + NR;
  constexpr int COQ = (CO + 3) / 4;
  constexpr int DP = 4 * COQ;                    // dY floats per pixel in LDS
  constexpr int XP = CSW;                        // X floats per halo pixel in LDS
  constexpr int LPX = (kTH + 2) * kLW;           // halo pixels
  // LDS floats per halo row: padded to = CSW (mod 16), so the 16 columns of a group -- (dh, ci)
  // runs crossing a dh boundary -- fall on 16 distinct banks mod 16; lane groups g and g + 1
  // are 4 pixels = 16 banks apart (4 XP = 16 mod 32), so a 32-lane half of a ds_read_b32
  // hits 32 distinct banks (the unpadded rows, = 8 mod 16, made 2-way conflicts in every
  // group that crosses a row)
  constexpr int RS = kLW * XP + ((CSW - kLW * XP) % 16 + 16) % 16;
  constexpr int G = (3 * CSW + 15) / 16;         // 16-column groups per dw
  constexpr int WCOL = NW / WPIX;
  constexpr int NT = 64 * NW;
  constexpr int GW = (G + WCOL - 1) / WCOL;      // groups per wave
  static_assert(NR <= 4 && (NR == 0 || COQ == 4 * TM + 1), "one remainder quad");
  static_assert(WCOL * WPIX == NW && (WCOL == 1 || WCOL == 2 || WCOL == 4), "waves per tile");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* xs = sm;                   // [kTH + 2][RS]: halo rows of kLW pixels x XP
  float* ds = sm + (kTH + 2) * RS;  // [kNPX][DP]

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int wc = wave % WCOL, wp = wave / WCOL;
  const int cis = blockIdx.y % p.n_ci_slabs, cos = blockIdx.y / p.n_ci_slabs;
  const int c0 = cis * CSW, co0 = cos * CO;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const __amdgpu_buffer_rsrc_t dr = make_rsrc(p.dy, p.dy_bytes);

  // this lane's column of each of the wave's groups: halo offset of (dh, ci) (an invalid
  // column reads the address of the last real one -- a broadcast, no bank conflict -- and
  // its sums are never written)
  int xoff[GW];
  bool colok[GW];
#pragma unroll
  for (int j = 0; j < GW; ++j) {
    const int n = (wc * GW + j) * 16 + r;
    const int nc = n < 3 * CSW ? n : 3 * CSW - 1;
    const int dh = nc / CSW, ci = nc - dh * CSW;
    colok[j] = wc * GW + j < G && n < 3 * CSW && c0 + ci < p.cin;
    xoff[j] = dh * RS + ci;
  }
  // input BatchNorm: the slab's scale / shift in LDS (read after the tile loop's first
  // barrier), applied to in-image pixels in the staging (= bn_apply_body's arithmetic)
  __shared__ f4 ibn_tab[2][CQ];
  if (p.isave && threadIdx.x < 2 * CSW) {
    const int k = threadIdx.x % CSW, which = threadIdx.x / CSW;
    const int ch = c0 + k < p.cin ? c0 + k : p.cin - 1;
    reinterpret_cast<float*>(&ibn_tab[which][0])[k] = p.isave[(2 + which) * p.cin + ch];
  }
  auto ibn = [&](f4& v, int q) {
    const f4 sc = ibn_tab[0][q], sh = ibn_tab[1][q];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float t = __builtin_fmaf(v[k], sc[k], sh[k]);
      v[k] = (p.irelu && t < 0.f) ? 0.f : t;
    }
  };

  f4 acc[TM][GW][3];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < GW; ++j)
#pragma unroll
      for (int d = 0; d < 3; ++d) acc[i][j][d] = f4{0.f, 0.f, 0.f, 0.f};
  float racc[GW][3][NR > 0 ? NR : 1];
#pragma unroll
  for (int j = 0; j < GW; ++j)
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
      for (int q = 0; q < NR; ++q) racc[j][d][q] = 0.f;

  const int per_img = p.tiles_h * p.tiles_w;
  const int tb = blockIdx.x * p.tps;
  const int te = tb + p.tps < p.ntiles ? tb + p.tps : p.ntiles;
  // staging map: thread -> one channel quad (fixed) and pixels b, b + XPU, b + 2 XPU, ...
  // (no per-item division by the quad count)
  constexpr int XPU = NT / CQ, DPU = NT / COQ;  // pixels per pass
  constexpr int NXI = (LPX + XPU - 1) / XPU, NDI = (kNPX + DPU - 1) / DPU;
  const int xq = threadIdx.x % CQ, xb = threadIdx.x / CQ;     // xb < XPU: active
  const int dq = threadIdx.x % COQ, db = threadIdx.x / COQ;
  const bool xact = xb < XPU, dact = db < DPU;
  const int xc = c0 + 4 * xq;
  const bool xcok = xc < p.cin4;
  const bool dcok = co0 + 4 * dq < p.cout;
  f4 px[NXI], pd[NDI];
  uint32_t xin = 0;  // in-image X items (input BatchNorm)
  auto fetch = [&](int tile) {
    const int img = (int)p.per_img_div.div((uint32_t)tile);
    const int trem = tile - img * per_img;
    const int th = (int)p.tiles_w_div.div((uint32_t)trem);
    const int oh0 = th * kTH, ow0 = (trem - th * p.tiles_w) * kTW;
    const int ibase = img * p.h;
#pragma unroll
    for (int u = 0; u < NXI; ++u) {
      const int hp = xb + u * XPU;
      const int lr = hp / kLW, lc = hp - lr * kLW;
      const int ih = oh0 - 1 + lr, iw = ow0 - 1 + lc;
      const bool ok = xact && hp < LPX && xcok && (unsigned)ih < (unsigned)p.h &&
                      (unsigned)iw < (unsigned)p.w;
      px[u] = load4(xr, ok ? (uint32_t)(((ibase + ih) * p.w + iw) * p.x_ps + xc) * 4u : kOOB);
      xin = u == 0 ? (uint32_t)ok : (xin | ((uint32_t)ok << u));
    }
#pragma unroll
    for (int u = 0; u < NDI; ++u) {
      const int pp = db + u * DPU;
      const int oh = oh0 + pp / kTW, ow = ow0 + (pp & (kTW - 1));
      const bool ok = dact && pp < kNPX && dcok && oh < p.h && ow < p.w;
      pd[u] = load4(dr, ok ? (uint32_t)(((ibase + oh) * p.w + ow) * p.dy_ps + co0 + 4 * dq) * 4u : kOOB);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < NXI; ++u) {
      const int hp = xb + u * XPU;
      if (!xact || hp >= LPX) break;
      f4 v = px[u];
      if (p.isave && ((xin >> u) & 1u)) ibn(v, xq);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = xc + k < p.cin ? v[k] : 0.f;  // channel padding
      const int lr = hp / kLW, lc = hp - lr * kLW;
      *reinterpret_cast<f4*>(&xs[lr * RS + lc * XP + 4 * xq]) = v;
    }
#pragma unroll
    for (int u = 0; u < NDI; ++u) {
      const int pp = db + u * DPU;
      if (!dact || pp >= kNPX) break;
      f4 v = pd[u];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = (co0 + 4 * dq + k < p.cout && 4 * dq + k < CO) ? v[k] : 0.f;
      *reinterpret_cast<f4*>(&ds[pp * DP + 4 * dq]) = v;
    }
  };

  if (PF && tb < te) fetch(tb);
  for (int tile = tb; tile < te; ++tile) {
    __syncthreads();  // the previous tile's reads are done
    if (!PF) fetch(tile);
    store();
    __syncthreads();
    if (PF && tile + 1 < te) fetch(tile + 1);
#pragma unroll 1
    for (int ch = wp; ch < kTH * 2; ch += WPIX) {
      const int orow = ch >> 1, cb = (ch & 1) * 16;
      const int dpx = orow * kTW + cb + 4 * g;  // first of this lane group's 4 pixels
      // A: 4 pixels x co (16 i + r); remainder rows: one quad per pixel (broadcast)
      float a[TM][4];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int s = 0; s < 4; ++s) a[i][s] = ds[(dpx + s) * DP + 16 * i + r];
      f4 rq[4];
      if constexpr (NR > 0) {
#pragma unroll
        for (int s = 0; s < 4; ++s) rq[s] = *reinterpret_cast<const f4*>(&ds[(dpx + s) * DP + 16 * TM]);
      }
      const int xb = orow * RS + (cb + 4 * g) * XP;
#pragma unroll
      for (int j = 0; j < GW; ++j) {
        float xv[6];
#pragma unroll
        for (int t = 0; t < 6; ++t) xv[t] = xs[xb + xoff[j] + t * XP];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < TM; ++i)
              acc[i][j][d] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], xv[d + s], acc[i][j][d], 0, 0, 0);
          if constexpr (NR > 0) {
#pragma unroll
            for (int q = 0; q < NR; ++q)
#pragma unroll
              for (int s = 0; s < 4; ++s) racc[j][d][q] = __builtin_fmaf(rq[s][q], xv[d + s], racc[j][d][q]);
          }
        }
      }
    }
  }

  // remainder rows: the 4 lane groups' pixel shares (fixed order)
#pragma unroll
  for (int j = 0; j < GW; ++j)
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
      for (int q = 0; q < NR; ++q) {
        float v = racc[j][d][q];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        racc[j][d][q] = v;
      }
  const int ncol4 = 9 * p.cin4;
  // part[split][co][col]: this block's slab through a buffer resource (32-bit offsets)
  const uint32_t slab = (uint32_t)(p.cout * ncol4);
  const __amdgpu_buffer_rsrc_t orr = make_rsrc(p.part + (int64_t)blockIdx.x * slab, slab * 4u);
  int colb[GW];  // column of (dh, ci) at dw = 0, or -1
#pragma unroll
  for (int j = 0; j < GW; ++j) {
    const int n = (wc * GW + j) * 16 + r;
    const int dh = n / CSW, ci = n - dh * CSW;
    colb[j] = colok[j] ? dh * 3 * p.cin4 + c0 + ci : -1;
  }
  auto write = [&](int j, int d, int i, int e, float v) {
    const int co = co0 + 16 * i + 4 * g + e;
    const bool ok = colb[j] >= 0 && co < p.cout;
    store1(orr, ok ? (uint32_t)(co * ncol4 + colb[j] + d * p.cin4) * 4u : kOOB, v);
  };
  auto write_r = [&](int j, int d, int q, float v) {
    const int co = co0 + 16 * TM + q;
    const bool ok = g == 0 && colb[j] >= 0 && co < p.cout;
    store1(orr, ok ? (uint32_t)(co * ncol4 + colb[j] + d * p.cin4) * 4u : kOOB, v);
  };
  if constexpr (WPIX == 1) {
#pragma unroll
    for (int j = 0; j < GW; ++j)
#pragma unroll
      for (int d = 0; d < 3; ++d) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) write(j, d, i, e, acc[i][j][d][e]);
#pragma unroll
        for (int q = 0; q < NR; ++q) write_r(j, d, q, racc[j][d][q]);
      }
  } else {
    // waves wp = 1 .. WPIX-1 hand their sums to wave wp = 0 of the same columns through LDS
    // (the staging tiles are no longer read), summed in wave order
    constexpr int NV = TM * GW * 3 * 4 + GW * 3 * NR;  // values per lane
    __syncthreads();
    float* red = sm;  // [WPIX-1][WCOL][NV][64]
    if (wp > 0) {
      float* o = red + ((wp - 1) * WCOL + wc) * NV * 64 + lane;
      int k = 0;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < GW; ++j)
#pragma unroll
          for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int e = 0; e < 4; ++e) o[64 * k++] = acc[i][j][d][e];
#pragma unroll
      for (int j = 0; j < GW; ++j)
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
          for (int q = 0; q < NR; ++q) o[64 * k++] = racc[j][d][q];
    }
    __syncthreads();
    if (wp == 0) {
#pragma unroll 1
      for (int w = 1; w < WPIX; ++w) {
        const float* o = red + ((w - 1) * WCOL + wc) * NV * 64 + lane;
        int k = 0;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < GW; ++j)
#pragma unroll
            for (int d = 0; d < 3; ++d)
#pragma unroll
              for (int e = 0; e < 4; ++e) acc[i][j][d][e] += o[64 * k++];
#pragma unroll
        for (int j = 0; j < GW; ++j)
#pragma unroll
          for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int q = 0; q < NR; ++q) racc[j][d][q] += o[64 * k++];
      }
#pragma unroll
      for (int j = 0; j < GW; ++j)
#pragma unroll
        for (int d = 0; d < 3; ++d) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) write(j, d, i, e, acc[i][j][d][e]);
#pragma unroll
          for (int q = 0; q < NR; ++q) write_r(j, d, q, racc[j][d][q]);
        }
    }
  }
}

namespace {

struct Cfg {
  int cq, tm, nr, wpix, ci_slabs, co_slabs;
  int pf = 0;
  int nw = 4;  // waves per workgroup
};

// 18 = 16 + 2 (one ci slab of 5 quads; 2 waves per column half of the tile's chunks); 36 = 32 + 4 (9 quads); 72 = 2 co slabs x (32 + 4),
// 2 ci slabs of 9 quads.  Anything else: not handled (0).
bool pick(const vae2_act* xd, const vae2_act* dyd, Cfg& c) {
  if (xd->c != dyd->c) return false;
  if (dyd->c == 18) c = Cfg{5, 1, 2, 2, 1, 1};
  else if (dyd->c == 36) c = Cfg{9, 2, 4, 1, 1, 1};
  else if (dyd->c == 72) c = Cfg{9, 2, 4, 1, 2, 2};
  else return false;
  c.pf = g_wgrad_narrow == 2;  // (tune key 7 = 2: register prefetch of the next tile)
  if (g_wgrad_narrow == 3) {    // (key 7 = 3: 8 waves, the extra 4 splitting the pixels)
    c.nw = 8;
    c.wpix *= 2;
  }
  return true;
}

size_t lds_bytes(const Cfg& c) {
  const int CO = 16 * c.tm + c.nr, DP = 4 * ((CO + 3) / 4);
  const int csw = 4 * c.cq, rs = kLW * csw + ((csw - kLW * csw) % 16 + 16) % 16;  // = RS
  const size_t stage = ((size_t)(kTH + 2) * rs + (size_t)kNPX * DP) * sizeof(float);
  const int G = (3 * 4 * c.cq + 15) / 16, wcol = c.nw / c.wpix, gw = (G + wcol - 1) / wcol;
  const size_t nv = (size_t)c.tm * gw * 12 + (size_t)gw * 3 * c.nr;
  const size_t red = c.wpix > 1 ? (size_t)(c.wpix - 1) * wcol * nv * 64 * sizeof(float) : 0;
  return stage > red ? stage : red;
}

const void* kernel_of(const Cfg& c) {
  if (c.nw == 8)
    return c.cq == 5 ? reinterpret_cast<const void*>(wgrad3n_kernel<5, 1, 2, 4, false, 8>)
                     : reinterpret_cast<const void*>(wgrad3n_kernel<9, 2, 4, 2, false, 8>);
  if (c.cq == 5) return c.pf ? reinterpret_cast<const void*>(wgrad3n_kernel<5, 1, 2, 2, true>)
                             : reinterpret_cast<const void*>(wgrad3n_kernel<5, 1, 2, 2, false>);
  return c.pf ? reinterpret_cast<const void*>(wgrad3n_kernel<9, 2, 4, 1, true>)
              : reinterpret_cast<const void*>(wgrad3n_kernel<9, 2, 4, 1, false>);
}

int resident_per_cu(const Cfg& c) {
  static int cache[6] = {0, 0, 0, 0, 0, 0};
  const int k = (c.cq == 5 ? 0 : 1) + (c.nw == 8 ? 4 : 2 * c.pf);
  if (!cache[k]) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel_of(c), 64 * c.nw, lds_bytes(c)) !=
            hipSuccess || n < 1) {
      (void)hipGetLastError();
      n = 1;
    }
    cache[k] = n;
  }
  return cache[k];
}

struct Plan {
  Cfg c;
  int tiles_h, tiles_w, ntiles, tps, splits;
};

bool plan(const vae2_act* xd, const vae2_act* dyd, Plan& pl) {
  if (g_bf16 || !g_wgrad_narrow || !pick(xd, dyd, pl.c)) return false;
  pl.tiles_h = (int)ceil_div(dyd->h, kTH);
  pl.tiles_w = (int)ceil_div(dyd->w, kTW);
  pl.ntiles = (int)(dyd->n * pl.tiles_h * pl.tiles_w);
  const int gy = pl.c.ci_slabs * pl.c.co_slabs;
  // one round of resident workgroups, at least 2 tiles each (partial slabs are HBM traffic)
  int64_t want = (int64_t)256 * resident_per_cu(pl.c) / gy;
  if (want < 1) want = 1;
  pl.tps = (int)ceil_div(pl.ntiles, want);
  if (pl.tps < g_wgrad_narrow_tps) pl.tps = g_wgrad_narrow_tps;
  pl.splits = (int)ceil_div(pl.ntiles, pl.tps);
  return true;
}

}  // namespace

// Partial-slab rows (splits) the narrow kernel writes for this layer, 0 when it does not
// apply (conv.hip sizes the workspace with the larger of the two forms).
int64_t wgrad3n_splits(const vae2_act* xd, const vae2_act* dyd) {
  Plan pl;
  return plan(xd, dyd, pl) ? pl.splits : 0;
}

// Launches the narrow kernel into part ([splits][cout][9 * cin4]); returns the number of
// splits written, 0 when the layer is not handled here, < 0 on a launch error.
int wgrad3n_launch(const float* x, const vae2_act* xd, const float* dy, const vae2_act* dyd,
                   float* part, const float* isave, int irelu, uint32_t x_bytes,
                   uint32_t dy_bytes, hipStream_t s) {
  Plan pl;
  if (!plan(xd, dyd, pl)) return 0;
  WGN p{};
  p.x = x; p.x_ps = (int)xd->ps; p.cin = (int)xd->c; p.cin4 = (int)((xd->c + 3) / 4 * 4);
  p.h = (int)xd->h; p.w = (int)xd->w;
  p.dy = dy; p.dy_ps = (int)dyd->ps; p.cout = (int)dyd->c;
  p.tiles_h = pl.tiles_h; p.tiles_w = pl.tiles_w; p.ntiles = pl.ntiles; p.tps = pl.tps;
  p.n_ci_slabs = pl.c.ci_slabs;
  p.per_img_div = FastDiv((uint32_t)(pl.tiles_h * pl.tiles_w));
  p.tiles_w_div = FastDiv((uint32_t)pl.tiles_w);
  p.x_bytes = x_bytes; p.dy_bytes = dy_bytes;
  p.part = part;
  p.isave = isave; p.irelu = irelu ? 1 : 0;
  dim3 grid((unsigned)pl.splits, (unsigned)(pl.c.ci_slabs * pl.c.co_slabs));
  const size_t shm = lds_bytes(pl.c);
  if (pl.c.cq == 5) {
    if (pl.c.nw == 8) VAE2_LAUNCH((wgrad3n_kernel<5, 1, 2, 4, false, 8>), grid, dim3(512), shm, s, p);
    else if (pl.c.pf) VAE2_LAUNCH((wgrad3n_kernel<5, 1, 2, 2, true>), grid, dim3(256), shm, s, p);
    else VAE2_LAUNCH((wgrad3n_kernel<5, 1, 2, 2, false>), grid, dim3(256), shm, s, p);
  } else {
    if (pl.c.nw == 8) VAE2_LAUNCH((wgrad3n_kernel<9, 2, 4, 2, false, 8>), grid, dim3(512), shm, s, p);
    else if (pl.c.pf) VAE2_LAUNCH((wgrad3n_kernel<9, 2, 4, 1, true>), grid, dim3(256), shm, s, p);
    else VAE2_LAUNCH((wgrad3n_kernel<9, 2, 4, 1, false>), grid, dim3(256), shm, s, p);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? pl.splits : -(int)e;
}

}  // namespace vae2
