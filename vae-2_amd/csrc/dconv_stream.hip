// Streaming direct 3x3 stride-1 convolution for the narrow HRNet branches: 18 -> 18 and
// 36 -> 36 channels (enc_hrnet.py:27-30 conv3x3 inside BasicBlock, :33-62), forward and
// data gradient (the transposed conv, weights packed mode 1 and taps flipped).
//
// dconv3_kernel (conv.hip) gives each workgroup one 8 x 32 output tile: it stages the
// 10 x 34 halo tile, waits, runs the MFMA loop, writes, and exits -- at 18 channels the
// staging, the barrier and the epilogue are a third of the kernel, never overlapped with
// the matrix cores, and the halo rows are loaded twice (1.33x the input bytes).  Here a
// workgroup owns a BAND of a 32-column strip and walks it 4 output rows per step:
//
//   * LDS holds a ring of 10 halo rows (34 pixels x all channel quads; rows of the band
//     start at ring slot (halo row) % 10); every step adds the 4 rows the next step needs,
//     so each input row is staged once per band (1.06x input bytes at 128 x 256);
//   * the next step's 4 rows are loaded into registers at the top of a step and written
//     into the ring after its MFMAs (global latency hidden behind the matrix cores), one
//     barrier per step: the slots they overwrite held rows the previous step used last;
//   * wave w computes output row 4s + w of step s (TM = 2 tiles of 16 pixels), K in the
//     (dh, dw, quad) order with every kernel row dh padded to whole 4-step chunks: the ring
//     row of a chunk is one value per (step, dh) and a lane's (dw, quad) column offset in
//     chunk c is the same for every dh (CPD registers set up once) -- no per-chunk index
//     arithmetic; as in dconv3_body, lane group g takes K step 4c + g of chunk c (A: one
//     ds_read_b128 from the ring; B: one 16-byte load of the packed weights, or from LDS
//     at set_tune key 11) and the last NR = 2 / 4 channels run on the VALU against the same
//     A fragments, two channels per v_pk_fma_f32 (their weights in LDS);
//   * the epilogue is branch-free: 32-bit buffer offsets from hoisted per-lane column
//     terms, out-of-range pixels masked with kOOB (loads return 0, stores drop);
//   * BatchNorm partial statistics accumulate in registers over the whole band and are
//     written once per workgroup (one partial row per workgroup: vae2_conv2d_fwd_stats_rows
//     reports the band count).
//
// The fused BatchNorm forms of dconv3_body carry over (BNX 1: relu?(x*scale + shift) of
// the producer BatchNorm applied in the staging, zero halo kept zero; BNX 2: the producer
// BatchNorm's backward partials (sum g, sum g*xhat) in the epilogue instead of (sum, sum^2)).
#include <type_traits>

#include "common.h"

namespace vae2 {

typedef float f2 __attribute__((ext_vector_type(2)));

int g_dconv_stream = 3;      // vae2_conv2d_set_tune key 9: bit 0 18 channels, bit 1 36 channels
int g_dconv_stream_wpc = 0;  // vae2_conv2d_set_tune key 10: target workgroups per CU (0 auto)
int g_dconv_stream_bl = 0;   // vae2_conv2d_set_tune key 11: 18-channel weights in LDS
int g_dconv_stream_spb = 1;  // vae2_conv2d_set_tune key 17: minimum 4-row steps per band (1 or 2;
                             // 1 since round 6: the 36-channel layers get 512 one-step bands
                             // instead of 256 two-step ones, step +0.5 %, scripts/gpu_r6_r.sh, _s.sh)

struct DStream {
  const float* a;
  int a_ps, a_c, img_h, img_w;
  int tiles_w, nbands, band_rows;  // strips per image row, bands per strip, rows per band
  const float* w;                  // packed [Npad][9][4Q] (mode 0, or mode 1 for FLIP)
  uint32_t a_bytes, w_bytes;
  int n;
  const float* bias;
  float* y;
  int y_ps;
  uint32_t y_bytes;  // y extent for the range-checked loads / stores
  float beta;
  float* stats;  // [2][gridDim.x][n] or null
  const float* isave;
  int irelu;
  const float* bx;
  int bx_ps, brelu;
  const float* bsave;
  uint32_t bx_bytes;
  int vec_out;  // y 16-byte aligned and y_ps % 4 == 0: quad-transposed 16-byte stores
};

constexpr int kDsRing = 10;  // halo rows resident in LDS
constexpr int kDsLW = 34;    // halo columns of a 32-column strip

// (exported symbol: the launch log names kernels through the dynamic symbol table)
template <int TN, int NR, int Q, bool FLIP, int BNX, bool BL>
__global__ __launch_bounds__(256, Q == 5 ? 4 : 1) void dconv3s_kernel(DStream p) {
  constexpr int TM = 2, LW = kDsLW, RING = kDsRing;
  constexpr int CSP = 4 * Q + 4;               // LDS floats per pixel (+4: bank spread)
  constexpr int RS = LW * CSP;                 // LDS floats per ring row
  constexpr int C4 = 4 * Q;                    // packed channels per tap
  constexpr int BN = 16 * TN, BNT = BN + NR;
  // K order (dh, dw, q), every kernel row dh padded to KD = whole 4-step chunks: chunk c
  // of row dh holds steps dh * KD + 4 c .. + 3, so the ring row of a chunk is one per-row
  // value and a lane's (dw, q) column offset in chunk c is the same for every row
  constexpr int KD = (3 * Q + 3) / 4 * 4, CPD = KD / 4, NK = 3 * KD;
  constexpr int PP = 256 / Q;                  // pixels per staging pass
  constexpr int NPF = (4 * LW + PP - 1) / PP;  // staged quads per thread per step
  constexpr int NPRO = (6 * LW + PP - 1) / PP;
  constexpr int NRP = NR / 2;                  // remainder channel pairs (packed FMAs)
  static_assert(NR == 2 || NR == 4, "remainder shape");
  static_assert(BNX == 0 || (BNX == 1) != FLIP, "input BN: forward; partials: dgrad");
  __shared__ __attribute__((aligned(16))) float ring[RING * RS];
  // remainder weights, step-major: rwp[k][jp][h] = (w[2jp][2h], w[2jp+1][2h], w[2jp][2h+1],
  // w[2jp+1][2h+1]) of step k's 4 channels -- the operand pairs of v_pk_fma_f32
  __shared__ f4 rwp[NK * NRP * 2];
  // BL (18 channels): the B operand from LDS as well (wl[k][n]) -- the main loop then
  // issues no global load, so waiting on a weight fragment never waits on the next rows'
  // staging loads too (vmcnt retires in order); 36 channels: 45 KB of weights would cost
  // 2 -> 1 blocks per CU, B stays a 16-byte global load
  __shared__ f4 wl[BL ? NK * BN : 1];
  __shared__ float red[4][2][BNT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int band = bid % p.nbands, t2 = bid / p.nbands;
  const int strip = t2 % p.tiles_w, img = t2 / p.tiles_w;
  const int oh0 = band * p.band_rows, ow0 = strip * 32;
  const int rows = min(p.band_rows, p.img_h - oh0);
  const int nsteps = (rows + 3) >> 2;
  const int img_base = img * p.img_h;
  const __amdgpu_buffer_rsrc_t arsrc = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t wrsrc = make_rsrc(p.w, p.w_bytes);

  // step k -> (tap t, quad q), valid = a real step (else zero weights)
  auto step_of = [](int k, int& t, int& q) {
    const int dh = k / KD, wk = k - dh * KD;
    const bool v = wk < 3 * Q;
    const int dw = v ? wk / Q : 0;
    q = v ? wk - dw * Q : 0;
    t = dh * 3 + dw;
    return v;
  };
  if constexpr (BL) {
    for (int i = tid; i < NK * BN; i += 256) {
      const int k = i / BN, n = i - k * BN;
      int t, q;
      const bool v = step_of(k, t, q);
      const int tl = FLIP ? 8 - t : t;
      wl[i] = v ? *reinterpret_cast<const f4*>(p.w + (int64_t)n * 9 * C4 + tl * C4 + 4 * q)
                : f4{0.f, 0.f, 0.f, 0.f};
    }
  }
  for (int i = tid; i < NK * NRP * 2; i += 256) {
    const int k = i / (NRP * 2), jp = (i >> 1) % NRP, h = i & 1;
    int t, q;
    const bool v = step_of(k, t, q);
    const int tl = FLIP ? 8 - t : t;
    const float* w0 = p.w + (int64_t)(BN + 2 * jp) * 9 * C4 + tl * C4 + 4 * q + 2 * h;
    const float* w1 = w0 + 9 * C4;
    rwp[i] = v ? f4{w0[0], w1[0], w0[1], w1[1]} : f4{0.f, 0.f, 0.f, 0.f};
  }
  // this lane's per-chunk (dw, q) column offsets (16-byte units) and, B from global, weight
  // byte offsets of row dh = 0 (row dh adds dh * 3 taps, FLIP: subtracts)
  int colofs[CPD];
  uint32_t wofs[BL ? 1 : CPD];
#pragma unroll
  for (int c = 0; c < CPD; ++c) {
    int t, q;
    const bool v = step_of(4 * c + g, t, q);
    colofs[c] = (t % 3) * (CSP / 4) + q;
    if constexpr (!BL) {
      const int tl = FLIP ? 8 - t : t;
      wofs[c] = v ? (uint32_t)(tl * C4 + 4 * q) * 4u : kOOB;
    }
  }

  // ---- staging: thread -> (channel quad sq, pixels pb + u * PP of a row group) ----
  const int sq = tid % Q, pb = tid / Q;
  const bool stager = pb < PP;
  const int cq = 4 * sq;
  const bool cpad = cq + 4 > p.a_c;
  f4 isc, ish;
  if (BNX == 1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int ch = cq + k < p.a_c ? cq + k : p.a_c - 1;
      isc[k] = p.isave[2 * p.a_c + ch];
      ish[k] = p.isave[3 * p.a_c + ch];
    }
  }
  // halo row hr of the band = input row oh0 - 1 + hr
  auto in_pix = [&](int hr0, int P, int& ih, int& iw) {
    const int lr = P / LW, lc = P - lr * LW;
    ih = oh0 - 1 + hr0 + lr;
    iw = ow0 - 1 + lc;
    return (unsigned)ih < (unsigned)p.img_h && (unsigned)iw < (unsigned)p.img_w;
  };
  // (cnt: std::integral_constant, so the register arrays are indexed at compile time)
  auto fetch = [&, arsrc](int hr0, int nrows, f4* v, auto cnt) {
#pragma unroll
    for (int u = 0; u < decltype(cnt)::value; ++u) {
      const int P = pb + u * PP;
      int ih, iw;
      const bool ok = stager && P < nrows * LW && in_pix(hr0, P, ih, iw);
      v[u] = load4(arsrc, ok ? (uint32_t)(((img_base + ih) * p.img_w + iw) * p.a_ps + cq) * 4u
                             : kOOB);
    }
  };
  auto put = [&](int hr0, int nrows, f4* v, auto cnt) {
#pragma unroll
    for (int u = 0; u < decltype(cnt)::value; ++u) {
      const int P = pb + u * PP;
      if (!stager || P >= nrows * LW) continue;
      int ih, iw;
      const bool ok = in_pix(hr0, P, ih, iw);
      f4 x = v[u];
      if (BNX == 1 && ok) {  // = bn_apply_body's arithmetic
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float t = __builtin_fmaf(x[k], isc[k], ish[k]);
          x[k] = (p.irelu && t < 0.f) ? 0.f : t;
        }
      }
      if (cpad) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (cq + k >= p.a_c) x[k] = 0.f;
      }
      const int lr = P / LW, lc = P - lr * LW;
      const int slot = (hr0 + lr) % RING;
      *reinterpret_cast<f4*>(&ring[slot * RS + lc * CSP + cq]) = x;
    }
  };
  {
    f4 pro[NPRO];
    fetch(0, 6, pro, std::integral_constant<int, NPRO>{});
    put(0, 6, pro, std::integral_constant<int, NPRO>{});
  }
  __syncthreads();

  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) abase[i] = (16 * i + r) * (CSP / 4);  // 16-byte units
  uint32_t wrow[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) wrow[j] = (uint32_t)((j * 16 + r) * 9 * C4) * 4u;

  float csum[TN], csq[TN], rsum[1], rsq[1];  // rsum / rsq: the group's remainder channel
  // producer BatchNorm (BNX 2): per-column mean, invstd, scale, shift
  float bmn[TN], bis[TN], bsc[TN], bsh[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    csum[j] = 0.f;
    csq[j] = 0.f;
    if (BNX == 2) {
      const int n = j * 16 + r;
      bmn[j] = p.bsave[n]; bis[j] = p.bsave[p.n + n];
      bsc[j] = p.bsave[2 * p.n + n]; bsh[j] = p.bsave[3 * p.n + n];
    }
  }
  // the remainder channel this lane group writes (group g < NR: channel BN + g) and its
  // producer-BN coefficients; bias of the lane's MFMA columns and of that channel
  const bool rown = g < NR;
  const int rn = BN + (rown ? g : 0);
  float bias_m[TN], bias_r = 0.f, rbmn = 0.f, rbis = 0.f, rbsc = 0.f, rbsh = 0.f;
#pragma unroll
  for (int j = 0; j < TN; ++j) bias_m[j] = p.bias ? p.bias[j * 16 + r] : 0.f;
  if (p.bias) bias_r = p.bias[rn];
  if (BNX == 2) {
    rbmn = p.bsave[rn]; rbis = p.bsave[p.n + rn];
    rbsc = p.bsave[2 * p.n + rn]; rbsh = p.bsave[3 * p.n + rn];
  }
  rsum[0] = 0.f;
  rsq[0] = 0.f;
  const __amdgpu_buffer_rsrc_t bxr = make_rsrc(p.bx, BNX == 2 ? p.bx_bytes : 0u);
  const __amdgpu_buffer_rsrc_t yr = make_rsrc(p.y, p.y_bytes);
  const bool has_beta = p.beta != 0.f;
  // per-lane output column terms (elements) and in-image limits, hoisted out of the steps:
  // MFMA layout pixel 16 i + 4 g + e, transposed 16 i + 4 g + (r & 3), remainder 16 i + r
  const uint32_t yps = (uint32_t)p.y_ps, xps = BNX == 2 ? (uint32_t)p.bx_ps : 0u;
  const uint32_t ycol = (uint32_t)(ow0 + 4 * g) * yps, xcol = (uint32_t)(ow0 + 4 * g) * xps;
  const uint32_t ycolk = (uint32_t)(ow0 + 4 * g + (r & 3)) * yps;
  const uint32_t ycolr = (uint32_t)(ow0 + r) * yps, xcolr = (uint32_t)(ow0 + r) * xps;
  const int wl_m = p.img_w - ow0 - 4 * g, wl_k = wl_m - (r & 3), wl_r = p.img_w - ow0 - r;

  for (int s = 0; s < nsteps; ++s) {
    const bool pf = s + 1 < nsteps;
    f4 nxt[NPF];
    if (pf) fetch(4 * s + 6, 4, nxt, std::integral_constant<int, NPF>{});

    // ---- MFMA main loop: output row 4s + wave, halo rows 4s + wave + dh ----
    // ring row of the wave's first input row, in 16-byte units (row dh: + dh rows, wrapped)
    const int hoff = ((4 * s + wave) % RING) * (RS / 4);
    f4 acc[TM][TN];
    f2 racc[TM][NRP];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < NRP; ++j) racc[i][j] = f2{0.f, 0.f};
    }
    const f4* ring4 = reinterpret_cast<const f4*>(ring);
    f4 fa[TM], fb[TN];
    // chunk c of kernel row dh into (fa, fb)
    auto load = [&](int dh, int c, f4* A, f4* B) {
      int base = hoff + dh * (RS / 4);
      base -= base >= RING * (RS / 4) ? RING * (RS / 4) : 0;
      base += colofs[c];
#pragma unroll
      for (int i = 0; i < TM; ++i) A[i] = ring4[base + abase[i]];
      const int k = dh * KD + 4 * c + g;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (BL) {
          B[j] = wl[k * BN + j * 16 + r];
        } else {
          const int dt = FLIP ? -3 * dh : 3 * dh;
          B[j] = load4(wrsrc, wrow[j] + wofs[c] + (uint32_t)(dt * C4 * 4));
        }
      }
    };
    auto mma = [&](int dh, int c, const f4* A, const f4* B) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[i][k], B[j][k], acc[i][j], 0, 0, 0);
      // VALU remainder: this lane's K step against the A fragments it holds, two channels
      // per v_pk_fma_f32
      const int k = dh * KD + 4 * c + g;
#pragma unroll
      for (int jp = 0; jp < NRP; ++jp) {
        const f4 w01 = rwp[(k * NRP + jp) * 2], w23 = rwp[(k * NRP + jp) * 2 + 1];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          racc[i][jp] = __builtin_elementwise_fma(f2{A[i][0], A[i][0]}, f2{w01[0], w01[1]}, racc[i][jp]);
          racc[i][jp] = __builtin_elementwise_fma(f2{A[i][1], A[i][1]}, f2{w01[2], w01[3]}, racc[i][jp]);
          racc[i][jp] = __builtin_elementwise_fma(f2{A[i][2], A[i][2]}, f2{w23[0], w23[1]}, racc[i][jp]);
          racc[i][jp] = __builtin_elementwise_fma(f2{A[i][3], A[i][3]}, f2{w23[2], w23[3]}, racc[i][jp]);
        }
      }
    };
    load(0, 0, fa, fb);
#pragma unroll 1
    for (int dh = 0; dh < 3; ++dh) {
#pragma unroll
      for (int c = 0; c < CPD; ++c) {
        f4 na[TM], nb[TN];
        // the next chunk (row dh + 1's first after the last; past row 2: row 2 again, unused)
        if (c + 1 < CPD) load(dh, c + 1, na, nb);
        else load(dh < 2 ? dh + 1 : 2, 0, na, nb);
        mma(dh, c, fa, fb);
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = na[i];
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = nb[j];
      }
    }

    // ---- epilogue: lane (g, r) holds pixels 16 i + 4 g + e, channel 16 j + r ----
    // (32-bit byte offsets through buffer resources: an out-of-range pixel gets kOOB, its
    //  load returns 0 and its store is dropped -- no branches, no 64-bit address math)
    const int orow = 4 * s + wave;
    const bool rok = orow < rows;
    const uint32_t rowpix = (uint32_t)((img_base + oh0 + (rok ? orow : 0)) * p.img_w);
    const uint32_t ypix = rowpix * yps, xpix = rowpix * xps;
    // element offsets: lane column term (hoisted) + a wave-uniform column delta d
    auto yo_m = [&](int d, int n) { return (ypix + ycol + (uint32_t)d * yps + (uint32_t)n) * 4u; };
    auto xo_m = [&](int d, int n) { return (xpix + xcol + (uint32_t)d * xps + (uint32_t)n) * 4u; };
    // old outputs (beta) and producer pre-BN values (BNX 2), one batch of loads each
    float yo[TM][4][TN], xv[TM][4][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool pin = rok && 16 * i + e < wl_m;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          yo[i][e][j] = has_beta ? load1(yr, pin ? yo_m(16 * i + e, j * 16 + r) : kOOB) : 0.f;
          if (BNX == 2) xv[i][e][j] = load1(bxr, pin ? xo_m(16 * i + e, j * 16 + r) : kOOB);
        }
      }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool pin = rok && 16 * i + e < wl_m;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          float v = acc[i][j][e] + bias_m[j];
          if (has_beta) v = __builtin_fmaf(p.beta, yo[i][e][j], v);
          acc[i][j][e] = v;
          if (BNX == 2) {
            const float x = xv[i][e][j];
            const float gv = (p.brelu && !(__builtin_fmaf(x, bsc[j], bsh[j]) > 0.f)) ? 0.f : v;
            csum[j] += pin ? gv : 0.f;
            csq[j] += pin ? gv * (x - bmn[j]) * bis[j] : 0.f;
          } else {
            csum[j] += pin ? v : 0.f;
            csq[j] += pin ? v * v : 0.f;
          }
        }
      }
    if (p.vec_out) {
      const int k = r & 3, qc = 4 * (r >> 2);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bool pin = rok && 16 * i < wl_k;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          f4 v = acc[i][j];
          quad_transpose(v, k);
          store4(yr, pin ? (ypix + ycolk + (uint32_t)(16 * i) * yps + (uint32_t)(j * 16 + qc)) * 4u : kOOB, v);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool pin = rok && 16 * i + e < wl_m;
#pragma unroll
          for (int j = 0; j < TN; ++j) store1(yr, pin ? yo_m(16 * i + e, j * 16 + r) : kOOB, acc[i][j][e]);
        }
    }
    // VALU channels: the 4 lane groups' K shares summed; group g < NR writes channel BN + g
    float rac[TM][NR];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        rac[i][j] = racc[i][j >> 1][j & 1];
        rac[i][j] += __shfl_xor(rac[i][j], 16, 64);
        rac[i][j] += __shfl_xor(rac[i][j], 32, 64);
      }
    {
      float rv[TM], ro[TM], rx[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        float v = rac[i][0];
#pragma unroll
        for (int j = 1; j < NR; ++j) v = g == j ? rac[i][j] : v;
        rv[i] = v;
        const bool pin = rown && rok && 16 * i < wl_r;
        ro[i] = has_beta ? load1(yr, pin ? (ypix + ycolr + (uint32_t)(16 * i) * yps + rn) * 4u : kOOB) : 0.f;
        if (BNX == 2) rx[i] = load1(bxr, pin ? (xpix + xcolr + (uint32_t)(16 * i) * xps + rn) * 4u : kOOB);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bool pin = rown && rok && 16 * i < wl_r;
        float v = rv[i] + bias_r;
        if (has_beta) v = __builtin_fmaf(p.beta, ro[i], v);
        store1(yr, pin ? (ypix + ycolr + (uint32_t)(16 * i) * yps + rn) * 4u : kOOB, v);
        float s0, s1;
        if (BNX == 2) {
          const float x = rx[i];
          const float gv = (p.brelu && !(__builtin_fmaf(x, rbsc, rbsh) > 0.f)) ? 0.f : v;
          s0 = gv;
          s1 = gv * (x - rbmn) * rbis;
        } else {
          s0 = v;
          s1 = v * v;
        }
        rsum[0] += pin ? s0 : 0.f;  // (this lane's channel: rsum[0] of group g holds BN + g)
        rsq[0] += pin ? s1 : 0.f;
      }
    }

    if (pf) put(4 * s + 6, 4, nxt, std::integral_constant<int, NPF>{});
    __syncthreads();
  }

  // ---- the band's BatchNorm partial row (fixed order: lanes, then waves) ----
  if (p.stats) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      csum[j] += __shfl_xor(csum[j], 16, 64);
      csum[j] += __shfl_xor(csum[j], 32, 64);
      csq[j] += __shfl_xor(csq[j], 16, 64);
      csq[j] += __shfl_xor(csq[j], 32, 64);
    }
    if (g == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        red[wave][0][j * 16 + r] = csum[j];
        red[wave][1][j * 16 + r] = csq[j];
      }
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {  // over the group's 16 pixels r
      rsum[0] += __shfl_xor(rsum[0], o, 64);
      rsq[0] += __shfl_xor(rsq[0], o, 64);
    }
    if (r == 0 && rown) {
      red[wave][0][BN + g] = rsum[0];
      red[wave][1][BN + g] = rsq[0];
    }
    __syncthreads();
    for (int c = tid; c < BNT; c += 256) {
      const float s0 = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
      const float s1 = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
      p.stats[(int64_t)bid * p.n + c] = s0;
      p.stats[(int64_t)(gridDim.x + bid) * p.n + c] = s1;
    }
  }
}

namespace {

struct DsPlan {
  int q, tiles_w, band_rows, nbands;
  int64_t wgs;
};

bool ds_plan(const vae2_act* ad, const vae2_act* yd, DsPlan* pl) {
  const int Q = (int)((ad->c + 3) / 4), N = (int)yd->c;
  // set_tune key 9 bit 0: 18 channels, bit 1: 36 channels (default both).  At 64 x 128 x 8
  // the streaming 36 -> 36 conv runs 24.0 / 23.9 us (fwd / dgrad) against 26.0 / 25.6 for
  // dconv3_kernel; at 18 channels it is level in isolation (28.8 vs 28.9 us at 128 x 256 x 8,
  // global weights, 4 workgroups per CU: 16-column MFMAs leave it overhead-bound) but the
  // step gains with it: 897.6 / 903 / 906 frames/s with neither / 36 / both
  if (!((Q == 5 && N == 18 && (g_dconv_stream & 1)) || (Q == 9 && N == 36 && (g_dconv_stream & 2))))
    return false;
  if (ad->n != yd->n || ad->h != yd->h || ad->w != yd->w) return false;
  DsPlan d;
  d.q = Q;
  d.tiles_w = (int)ceil_div(yd->w, 32);
  const int64_t qsteps = ceil_div(yd->h, 4);
  const int64_t total = yd->n * d.tiles_w * qsteps;
  const int wpc = g_dconv_stream_wpc > 0 ? g_dconv_stream_wpc : (Q == 5 ? 4 : 2);
  int64_t spb = ceil_div(total, 256LL * wpc);
  if (spb < g_dconv_stream_spb) spb = g_dconv_stream_spb;
  if (spb > qsteps) spb = qsteps;
  d.band_rows = (int)(4 * spb);
  d.nbands = (int)ceil_div(yd->h, d.band_rows);
  d.wgs = yd->n * d.tiles_w * d.nbands;
  if (d.wgs >= (1LL << 31)) return false;
  if (pl) *pl = d;
  return true;
}

template <int TN, int NR, int Q, bool FLIP, bool BL>
void ds_launch_bnx(const DStream& p, dim3 grid, hipStream_t s) {
  if (FLIP && p.bx) VAE2_LAUNCH((dconv3s_kernel<TN, NR, Q, FLIP, FLIP ? 2 : 0, BL>), grid, dim3(256), 0, s, p);
  else if (!FLIP && p.isave) VAE2_LAUNCH((dconv3s_kernel<TN, NR, Q, FLIP, FLIP ? 0 : 1, BL>), grid, dim3(256), 0, s, p);
  else VAE2_LAUNCH((dconv3s_kernel<TN, NR, Q, FLIP, 0, BL>), grid, dim3(256), 0, s, p);
}

}  // namespace

bool dconv3s_shape(const vae2_act* ad, const vae2_act* yd) { return ds_plan(ad, yd, nullptr); }

int64_t dconv3s_rows(const vae2_act* ad, const vae2_act* yd) {
  DsPlan d;
  return ds_plan(ad, yd, &d) ? d.wgs : 0;
}

int dconv3s_launch(const float* a, const vae2_act* ad, const float* wp, uint32_t w_bytes,
                   const float* bias, float* y, const vae2_act* yd, float beta, float* stats,
                   bool flip, const float* isave, int irelu, const float* bx, int bx_ps,
                   int brelu, const float* bsave, uint32_t bx_bytes, uint32_t a_bytes,
                   hipStream_t s) {
  DsPlan d;
  if (!ds_plan(ad, yd, &d)) return 0;
  DStream p{};
  p.a = a; p.a_ps = (int)ad->ps; p.a_c = (int)ad->c;
  p.img_h = (int)ad->h; p.img_w = (int)ad->w;
  p.tiles_w = d.tiles_w; p.nbands = d.nbands; p.band_rows = d.band_rows;
  p.w = wp; p.a_bytes = a_bytes; p.w_bytes = w_bytes;
  p.n = (int)yd->c; p.bias = bias; p.y = y; p.y_ps = (int)yd->ps; p.beta = beta;
  // (the extent act_bytes in conv.hip gives: the last pixel's channels, its padded quad
  //  when the pixel stride is a multiple of 4)
  const int64_t ytail = (yd->ps % 4 == 0) ? (yd->c + 3) / 4 * 4 : yd->c;
  p.y_bytes = (uint32_t)(((yd->n * yd->h * yd->w - 1) * yd->ps + ytail) * 4);
  p.stats = stats;
  p.isave = isave; p.irelu = irelu;
  p.bx = bx; p.bx_ps = bx_ps; p.brelu = brelu; p.bsave = bsave; p.bx_bytes = bx_bytes;
  p.vec_out = ((uintptr_t)y % 16 == 0) && (yd->ps % 4 == 0);
  const dim3 grid((unsigned)d.wgs);
  if (d.q == 5 && g_dconv_stream_bl) {
    if (flip) ds_launch_bnx<1, 2, 5, true, true>(p, grid, s);
    else ds_launch_bnx<1, 2, 5, false, true>(p, grid, s);
  } else if (d.q == 5) {
    if (flip) ds_launch_bnx<1, 2, 5, true, false>(p, grid, s);
    else ds_launch_bnx<1, 2, 5, false, false>(p, grid, s);
  } else {
    if (flip) ds_launch_bnx<2, 4, 9, true, false>(p, grid, s);
    else ds_launch_bnx<2, 4, 9, false, false>(p, grid, s);
  }
  return 1;
}

}  // namespace vae2
