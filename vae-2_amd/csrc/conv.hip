// Convolutions of the HRNet stacks as implicit GEMMs on the fp32 matrix cores
// (v_mfma_f32_16x16x4_f32: exact fp32 FMA chains, 64 FLOP/clk/SIMD on gfx950).
//
//   forward     Y[m][n] = sum_k A[m][k] * B[k][n]
//               m = output pixel, n = Cout, k = (tap, Cin4); A = im2col(X) gathered
//               from NHWC on the fly, B = weights packed [Npad][k*k][Cin4].
//   bwd data    same kernel: m = input pixel of one stride-parity class per launch,
//               n = Cin, k = (valid tap, Cout4), A = dY gathered, B = weights packed
//               [Cin_pad][k*k][Cout4] (the transposed conv).
//   bwd weight  dW[co][(tap, ci)] = sum_p dY[p][co] * X[src(p, tap)][ci], split over
//               pixels into fp32 slabs (one per wave), then a fixed-order reduction
//               into the [Cout][Cin][kh][kw] gradient (deterministic).
//
// Fragment-direct loads: Cin is padded to a multiple of 4 (Cin4) inside K, and in
// each 16-deep K chunk lane group g = lane>>4 owns the 4 consecutive k = 4g..4g+3,
// i.e. 4 consecutive channels of ONE tap.  MFMA k-step s uses k = 4g+s for both
// operands (a permutation of the reduction order the sum does not see).  So a
// lane's A fragment for 4 k-steps is one 16-byte load of an NHWC pixel and its B
// fragment one 16-byte load of the packed weights: no LDS staging, no barriers in
// the main loop; fragments are double-buffered in registers.
//
// Replaces nn.Conv2d forward/backward for every conv of enc_hrnet.py (call sites
// in include/vae2_hip.h).
#include <mutex>
#include <vector>

#include "common.h"

// Diagnostic builds only (never the shipped library): -DVAE2_ABLATE=1 stages zeros
// instead of loading the direct kernel's halo tile, 2 drops its output stores, 4 skips its
// MFMA main loop (bits combine).
#ifndef VAE2_ABLATE
#define VAE2_ABLATE 0
#endif

// The build compiles this file once per part (-DVAE2_CONV_PART=0..3, in parallel): each
// part defines the host launchers of one kernel family, so the kernel templates are
// instantiated (and compiled) in that part only.  0: weight packing and the forward /
// data-gradient C ABI; 1: gather implicit GEMM; 2: direct 3x3 (+ grouped launches);
// 3: weight gradients.  Without the macro everything is in one translation unit.
#ifndef VAE2_CONV_PART
#define VAE2_CONV_PART -1
#endif
#define VAE2_PART(n) (VAE2_CONV_PART < 0 || VAE2_CONV_PART == (n))

namespace vae2 {


static inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

#if VAE2_PART(0)
// ------------------------------------------------------------ weight pack ----
// mode 0: out[n][t][c4] = w[n][c][t]         n < round_up(cout,64), c4 < round_up(cin,4)
// mode 1: out[n][t][c4] = w[c][n][t]         n < round_up(cin,64),  c4 < round_up(cout,4)
// (rows padded to 64 = the widest N tile, so B loads never need a bounds check).
// w[co][ci][t] lives at w[co*ld + ci*kk + t]: ld = cin*kk for a whole weight, larger
// for an input-channel block of a wider one (the per-branch blocks of a head conv).
__global__ void pack_weight_kernel(const float* __restrict__ w, int cout, int cin, int kk,
                                   int mode, int ld, float* __restrict__ out) {
  const int rows = mode == 0 ? (cout + 63) / 64 * 64 : (cin + 63) / 64 * 64;
  const int cols4 = mode == 0 ? (cin + 3) / 4 * 4 : (cout + 3) / 4 * 4;
  const int total = rows * kk * cols4;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    int n = i / (kk * cols4);
    int rem = i - n * kk * cols4;
    int t = rem / cols4;
    int c = rem - t * cols4;
    float v = 0.f;
    if (mode == 0) {
      if (n < cout && c < cin) v = w[(int64_t)n * ld + c * kk + t];
    } else {
      if (n < cin && c < cout) v = w[(int64_t)c * ld + n * kk + t];
    }
    out[i] = v;
  }
}

// One block row (blockIdx.y) per packing job.
__global__ __launch_bounds__(256) void pack_weights_batched_kernel(const vae2_pack_job* jobs) {
  const vae2_pack_job j = jobs[blockIdx.y];
  const int kk = j.k * j.k;
  const int rows = j.mode == 0 ? (j.cout + 63) / 64 * 64 : (j.cin + 63) / 64 * 64;
  const int cols4 = j.mode == 0 ? (j.cin + 3) / 4 * 4 : (j.cout + 3) / 4 * 4;
  const int per_row = kk * cols4;
  const int total = rows * per_row;
  const int64_t ld = j.ld > 0 ? j.ld : (int64_t)j.cin * kk;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int n = i / per_row;
    const int rem = i - n * per_row;
    const int t = rem / cols4;
    const int c = rem - t * cols4;
    float v = 0.f;
    if (j.mode == 0) {
      if (n < j.cout && c < j.cin) v = j.w[(int64_t)n * ld + c * kk + t];
    } else {
      if (n < j.cin && c < j.cout) v = j.w[(int64_t)c * ld + n * kk + t];
    }
    j.out[i] = v;
  }
}

#endif  // VAE2_PART(0)
// ------------------------------------------------------------ igemm ----
struct IGemm {
  const float* a;  // gathered activation (NHWC)
  int a_ps, a_c, a_c4, a_h, a_w;
  int g_n, g_h, g_w;  // iteration grid, M = g_n*g_h*g_w
  int a_step;         // A source row = g*a_step + d(tap)
  int nth, ntw;       // taps: t = th*ntw + tw
  int dh0, dhs, dw0, dws;
  int kh0, khs, kw0, kws, ksz;  // weight tap (kh0 + th*khs, kw0 + tw*kws) of a ksz x ksz kernel
  const float* w;               // packed [Npad][ksz*ksz][a_c4]
  uint32_t a_bytes, w_bytes;    // buffer extents for the range-checked loads
  int n;                        // GEMM N (real)
  const float* bias;
  float* y;
  int y_ps, y_h, y_w, y_step, y_offh, y_offw;
  float beta;
  float* stats;  // [2][gridDim.x][n] or null
  int vec_out;   // y 16-byte aligned, y_ps % 4 == 0, no statistics with beta != 0
  FastDiv hw_div, w_div;  // divide by g_h*g_w, g_w
  int ktab;               // use the K-step table (set_tune key 12, default on)
  // Data gradient (ROLE 1) with bx set (round 6): y is the gradient of a BatchNorm(+ReLU)
  // layer's output whose only consumer is this conv; the epilogue writes that layer's
  // backward partials (sum g, sum g*xhat; g = y masked by the ReLU recomputed from bx)
  // into stats, [2][gridDim.x * gridDim.z][n] (row = class * gridDim.x + tile), instead of
  // the layer's own reduce pass.  bx = its pre-BN tensor (y's pixels and channels).
  const float* bx;
  int bx_ps, brelu;
  const float* bsave;
  uint32_t bx_bytes;
  // Strided data gradient: one launch covers every stride-parity class of the input
  // pixels, class = blockIdx.z (gridDim.z == 1: the fields above are used as they are).
  struct Cls {
    int g_h, g_w, nth, ntw, dh0, dw0, kh0, kw0, y_offh, y_offw;
    FastDiv hw_div, w_div;
  } cls[4];
};

// KS = 4: in-workgroup K split for layers with too few row tiles to fill the chip: the 4
// waves share one (16*TM)-row tile, wave w takes K chunks w, w+4, ..., and the partial
// tiles are summed in LDS in a fixed order (deterministic) before wave 0's epilogue.
// NR > 0 (fp32, KS = 1, one N block): N = 16*TN + NR (18 = 16 + 2, 36 = 32 + 4) -- the
// last NR output channels on the VALU beside the MFMAs instead of a mostly-padding MFMA
// column tile: every lane already holds its A fragment (pixel r, 4 channels of the chunk),
// multiplies it with the remainder rows' weights for those channels, and the 4 lane
// groups' K shares are summed at the end (dconv3_kernel's remainder, for the gather GEMM).
constexpr int kIgTab = 1024;  // igemm K-step table entries (16 KB of LDS)

template <int TM, int TN, bool VEC, int ROLE, int KS = 1, bool BF = false, int NR = 0>
__global__ __launch_bounds__(256) void igemm_kernel(IGemm pin) {
  IGemm p = pin;
  if (gridDim.z > 1) {
    const IGemm::Cls& c = pin.cls[blockIdx.z];
    p.g_h = c.g_h; p.g_w = c.g_w; p.nth = c.nth; p.ntw = c.ntw;
    p.dh0 = c.dh0; p.dw0 = c.dw0; p.kh0 = c.kh0; p.kw0 = c.kw0;
    p.y_offh = c.y_offh; p.y_offw = c.y_offw; p.hw_div = c.hw_div; p.w_div = c.w_div;
  }
  constexpr int BN = 16 * TN;
  static_assert(NR == 0 || (KS == 1 && !BF && NR <= 4), "remainder form");
  __shared__ float red[4][2][BN + NR];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int M = p.g_n * p.g_h * p.g_w;
  const int bm = xcd_remap(blockIdx.x, gridDim.x);
  const int mw = (KS == 1 ? bm * 4 + wave : bm) * (16 * TM);
  const int n0 = blockIdx.y * BN;
  const int kk4 = p.ksz * p.ksz * p.a_c4;

  // this lane's A rows: m = mw + i*16 + r
  int rpix[TM], ri[TM], rj[TM];
  bool rok[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int m = mw + i * 16 + r;
    rok[i] = m < M;
    int mm = rok[i] ? m : 0;
    int gn = (int)p.hw_div.div((uint32_t)mm);
    int rem = mm - gn * p.g_h * p.g_w;
    int gi = (int)p.w_div.div((uint32_t)rem);
    int gj = rem - gi * p.g_w;
    ri[i] = gi * p.a_step;
    rj[i] = gj * p.a_step;
    rpix[i] = (gn * p.a_h + ri[i]) * p.a_w + rj[i];
  }
  // Buffer resources (wave-uniform): out-of-range offsets load 0, so padding taps,
  // rows past M and the K tail need no branches.
  const __amdgpu_buffer_rsrc_t arsrc = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t wrsrc = make_rsrc(p.w, p.w_bytes);
  uint32_t wrow[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) wrow[j] = (uint32_t)((n0 + j * 16 + r) * kk4) * 4u;
  uint32_t wrowr[NR > 0 ? NR : 1];  // remainder rows BN + q of the packed weights
#pragma unroll
  for (int q = 0; q < NR; ++q) wrowr[q] = (uint32_t)((n0 + BN + q) * kk4) * 4u;
  float racc[TM][NR > 0 ? NR : 1];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int q = 0; q < NR; ++q) racc[i][q] = 0.f;

  const int ntaps = p.nth * p.ntw;
  const int K = ntaps * p.a_c4;
  const int nchunks = KS == 1 ? (K + 15) >> 4 : (((K + 15) >> 4) + KS - 1 - wave) / KS;
  int tt = 0, c0 = 4 * g + (KS == 1 ? 0 : 16 * wave);
  while (c0 >= p.a_c4) { c0 -= p.a_c4; ++tt; }
  const bool cpad = (p.a_c & 3) != 0;
  // K-step table (quad step k = (tap, quad) of the linear K order): the tap decode (a
  // division by ntw), the carry loop and the tap's A / B offsets computed once per
  // workgroup instead of per lane and chunk; entry = (dh, dw | c0 << 16, weight byte
  // offset, A element offset (dh * a_w + dw) * a_ps + c0).  Steps past K (the prefetch of
  // the chunk pairs) get dh far outside the image and kOOB weights: zero operands.
  __shared__ int4 ktab[kIgTab];
  const int nq = K >> 2;                                  // quad steps
  // entries the loop can read: every wave's chunks + the 2 prefetched past its last
  const int nqt = 4 * ((K + 15) >> 4) + 16 * KS + 16;
  const bool use_tab = !BF && p.ktab && nqt <= kIgTab;
  if (use_tab) {
    const int q4 = p.a_c4 >> 2;
    for (int k = threadIdx.x; k < nqt; k += 256) {
      int4 e;
      if (k < nq) {
        const int t = k / q4, q = k - t * q4;
        const int th = t / p.ntw, tw = t - th * p.ntw;
        const int dh = p.dh0 + th * p.dhs, dw = p.dw0 + tw * p.dws;
        const int tlin = (p.kh0 + th * p.khs) * p.ksz + (p.kw0 + tw * p.kws);
        e = make_int4(dh, (dw & 0xffff) | (4 * q) << 16, (int)((uint32_t)(tlin * p.a_c4 + 4 * q) * 4u),
                      (dh * p.a_w + dw) * p.a_ps + 4 * q);
      } else {
        e = make_int4(1 << 20, 0, (int)kOOB, 0);
      }
      ktab[k] = e;
    }
  }
  __syncthreads();
  int kq = g + (KS == 1 ? 0 : 4 * wave);  // this lane's next quad step (as c0 / tt above)
  int rbase[TM];  // rpix * a_ps: the row's pixel in elements
#pragma unroll
  for (int i = 0; i < TM; ++i) rbase[i] = rpix[i] * p.a_ps;

  f4 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  f4 fr0[NR > 0 ? NR : 1], fr1[NR > 0 ? NR : 1];  // remainder weights of the chunk
  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  auto load = [&](f4* fa, f4* fb, f4* fr, int& mk) {
    if (use_tab) {
      const int4 e = ktab[kq];
      kq += 4 * KS;
      const int dh = e.x, dw = (int)(short)(e.y & 0xffff), cq = e.y >> 16;
      const uint32_t woff = (uint32_t)e.z;
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = load4(wrsrc, wrow[j] + woff);
#pragma unroll
      for (int q = 0; q < NR; ++q) fr[q] = load4(wrsrc, woff == kOOB ? kOOB : wrowr[q] + woff);
      const bool m1 = cq + 1 < p.a_c, m2 = cq + 2 < p.a_c, m3 = cq + 3 < p.a_c;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int ih = ri[i] + dh, iw = rj[i] + dw;
        const bool ok = rok[i] && (unsigned)ih < (unsigned)p.a_h && (unsigned)iw < (unsigned)p.a_w;
        const uint32_t off = ok ? (uint32_t)(rbase[i] + e.w) * 4u : kOOB;
        f4 v;
        if (VEC) {
          v = load4(arsrc, off);
        } else {
          v[0] = load1(arsrc, off);
          v[1] = load1(arsrc, m1 ? off + 4u : kOOB);
          v[2] = load1(arsrc, m2 ? off + 8u : kOOB);
          v[3] = load1(arsrc, m3 ? off + 12u : kOOB);
        }
        fa[i] = v;
      }
      mk = (m1 ? 2 : 0) | (m2 ? 4 : 0) | (m3 ? 8 : 0);
      return;
    }
    const bool tv = tt < ntaps;
    const int tc = tv ? tt : 0;
    const int th = tc / p.ntw;
    const int tw = tc - th * p.ntw;
    const int dh = p.dh0 + th * p.dhs, dw = p.dw0 + tw * p.dws;
    const int tlin = (p.kh0 + th * p.khs) * p.ksz + (p.kw0 + tw * p.kws);
    const uint32_t woff = tv ? (uint32_t)(tlin * p.a_c4 + c0) * 4u : kOOB;
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[j] = load4(wrsrc, wrow[j] + woff);
#pragma unroll
    for (int q = 0; q < NR; ++q) fr[q] = load4(wrsrc, tv ? wrowr[q] + woff : kOOB);
    const int doff = dh * p.a_w + dw;
    const bool m1 = c0 + 1 < p.a_c, m2 = c0 + 2 < p.a_c, m3 = c0 + 3 < p.a_c;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ih = ri[i] + dh, iw = rj[i] + dw;
      const bool ok = tv && rok[i] && (unsigned)ih < (unsigned)p.a_h &&
                      (unsigned)iw < (unsigned)p.a_w;
      const uint32_t off = ok ? (uint32_t)((rpix[i] + doff) * p.a_ps + c0) * 4u : kOOB;
      f4 v;
      if (VEC) {
        v = load4(arsrc, off);  // channel-pad lanes are masked where consumed (mma)
      } else {
        v[0] = load1(arsrc, off);
        v[1] = load1(arsrc, m1 ? off + 4u : kOOB);
        v[2] = load1(arsrc, m2 ? off + 8u : kOOB);
        v[3] = load1(arsrc, m3 ? off + 12u : kOOB);
      }
      fa[i] = v;
    }
    mk = (m1 ? 2 : 0) | (m2 ? 4 : 0) | (m3 ? 8 : 0);
    c0 += 16 * KS;
    while (c0 >= p.a_c4) { c0 -= p.a_c4; ++tt; }
  };
  // Masking the pad lanes here (not right after the loads) keeps the next chunk's
  // loads in flight across this chunk's MFMAs.
  auto mma = [&](f4* fa, const f4* fb, const f4* fr, int mk) {
    if (VEC && cpad) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        fa[i][1] = (mk & 2) ? fa[i][1] : 0.f;
        fa[i][2] = (mk & 4) ? fa[i][2] : 0.f;
        fa[i][3] = (mk & 8) ? fa[i][3] : 0.f;
      }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < NR; ++q)
#pragma unroll
        for (int s = 0; s < 4; ++s) racc[i][q] = __builtin_fmaf(fa[i][s], fr[q][s], racc[i][q]);
  };

  // Chunk pairs; the (possibly) extra odd chunk loads zeros (tt >= ntaps).
  if (mw < M && !BF) {
    int mk0 = 0, mk1 = 0;
    load(fa0, fb0, fr0, mk0);
    for (int ch = 0; ch < nchunks; ch += 2) {
      load(fa1, fb1, fr1, mk1);
      mma(fa0, fb0, fr0, mk0);
      load(fa0, fb0, fr0, mk0);
      mma(fa1, fb1, fr1, mk1);
    }
  } else if (mw < M) {  // bf16 operands: one 16x16x32 MFMA per chunk pair
    int mk0 = 0, mk1 = 0;
    load(fa0, fb0, fr0, mk0);
    load(fa1, fb1, fr1, mk1);
    for (int ch = 0; ch < nchunks; ch += 2) {
      if (VEC && cpad) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          fa0[i][1] = (mk0 & 2) ? fa0[i][1] : 0.f;
          fa0[i][2] = (mk0 & 4) ? fa0[i][2] : 0.f;
          fa0[i][3] = (mk0 & 8) ? fa0[i][3] : 0.f;
          fa1[i][1] = (mk1 & 2) ? fa1[i][1] : 0.f;
          fa1[i][2] = (mk1 & 4) ? fa1[i][2] : 0.f;
          fa1[i][3] = (mk1 & 8) ? fa1[i][3] : 0.f;
        }
      }
      bf16x8 A[TM], B[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) A[i] = pack_bf16(fa0[i], fa1[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) B[j] = pack_bf16(fb0[j], fb1[j]);
      load(fa0, fb0, fr0, mk0);
      load(fa1, fb1, fr1, mk1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], B[j], acc[i][j], 0, 0, 0);
    }
  }

  if constexpr (KS > 1) {
    __shared__ float kred[KS - 1][TM * TN * 4][64];
    if (wave > 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) kred[wave - 1][(i * TN + j) * 4 + e][lane] = acc[i][j][e];
    }
    __syncthreads();
    if (wave > 0) return;  // no barrier below on this path
#pragma unroll
    for (int w = 0; w < KS - 1; ++w)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][e] += kred[w][(i * TN + j) * 4 + e][lane];
  }

  // ---- epilogue ----
  float csum[TN], csq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) { csum[j] = 0.f; csq[j] = 0.f; }
  // producer BatchNorm backward partials (data gradient, bx set): per-column mean, invstd,
  // scale, shift of that layer (bn_bwd_reduce_body's arithmetic, element by element)
  constexpr bool BP = ROLE == 1 && !BF;
  const bool bnp = BP && p.bx != nullptr;
  float bmn[BP ? TN : 1], bis[BP ? TN : 1], bsc[BP ? TN : 1], bsh[BP ? TN : 1];
  if constexpr (BP) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + j * 16 + r < p.n ? n0 + j * 16 + r : p.n - 1;
      bmn[j] = bnp ? p.bsave[n] : 0.f;
      bis[j] = bnp ? p.bsave[p.n + n] : 0.f;
      bsc[j] = bnp ? p.bsave[2 * p.n + n] : 0.f;
      bsh[j] = bnp ? p.bsave[3 * p.n + n] : 0.f;
    }
  }
  // output pixel of GEMM row m (m < M)
  auto pix_of = [&](int m) {
    const int gn = (int)p.hw_div.div((uint32_t)m);
    const int rem = m - gn * p.g_h * p.g_w;
    const int gi = (int)p.w_div.div((uint32_t)rem);
    const int gj = rem - gi * p.g_w;
    return (gn * p.y_h + gi * p.y_step + p.y_offh) * p.y_w + gj * p.y_step + p.y_offw;
  };
  if (p.vec_out && (KS == 1 || wave == 0)) {
    // statistics in the MFMA layout (beta = 0 whenever they are requested), then each
    // 16x16 tile transposed inside lane quads: one 16-byte store per lane and tile, and
    // one output-pixel address per lane and row tile instead of four
    const int k = r & 3, qc = 4 * (r >> 2);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if (BP && bnp && p.stats) {
        // the row tile's 4 x TN pre-BN values, one batch of range-checked loads
        const __amdgpu_buffer_rsrc_t bxr = make_rsrc(p.bx, p.bx_bytes);
        float xv[4][TN];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int me = mw + i * 16 + g * 4 + e;
          const bool mok = me < M;
          const int pix = pix_of(mok ? me : 0);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int n = n0 + j * 16 + r;
            xv[e][j] = load1(bxr, mok && n < p.n ? (uint32_t)(pix * p.bx_ps + n) * 4u : kOOB);
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool mok = mw + i * 16 + g * 4 + e < M;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int n = n0 + j * 16 + r;
            const float v = acc[i][j][e];
            const float x = xv[e][j];
            const float gv = (p.brelu && !(__builtin_fmaf(x, bsc[j], bsh[j]) > 0.f)) ? 0.f : v;
            const bool ok = mok && n < p.n;
            csum[j] += ok ? gv : 0.f;
            csq[j] += ok ? gv * (x - bmn[j]) * bis[j] : 0.f;
          }
        }
      } else if (p.stats) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (mw + i * 16 + g * 4 + e >= M) continue;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int n = n0 + j * 16 + r;
            if (n >= p.n) continue;
            const float v = acc[i][j][e] + (p.bias ? p.bias[n] : 0.f);
            csum[j] += v;
            csq[j] += v * v;
          }
        }
      }
      const int m = mw + i * 16 + g * 4 + k;
      const bool mok = m < M;
      const int mm = mok ? m : 0;
      const int gn = (int)p.hw_div.div((uint32_t)mm);
      const int rem = mm - gn * p.g_h * p.g_w;
      const int gi = (int)p.w_div.div((uint32_t)rem);
      const int gj = rem - gi * p.g_w;
      float* yrow = p.y + ((gn * p.y_h + gi * p.y_step + p.y_offh) * p.y_w +
                           gj * p.y_step + p.y_offw) * p.y_ps;
      // beta: the row tile's old output quads all loaded before any store (one round trip
      // per row tile instead of one per quad: loads cannot pass the stores to y)
      f4 yold[TN];
      if (p.beta != 0.f) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + j * 16 + qc;
          yold[j] = (mok && n + 3 < p.n) ? *reinterpret_cast<const f4*>(yrow + n)
                                         : f4{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f4 v = acc[i][j];
        quad_transpose(v, k);
        const int n = n0 + j * 16 + qc;
        if (!mok || n >= p.n) continue;
        if (p.bias) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] += n + q < p.n ? p.bias[n + q] : 0.f;
        }
        if (n + 3 < p.n) {
          if (p.beta != 0.f) v += p.beta * yold[j];
          *reinterpret_cast<f4*>(yrow + n) = v;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (n + q < p.n) yrow[n + q] = p.beta != 0.f ? v[q] + p.beta * yrow[n + q] : v[q];
        }
      }
    }
  } else
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = mw + i * 16 + g * 4 + e;
      if (m >= M) continue;
      const int gn = (int)p.hw_div.div((uint32_t)m);
      const int rem = m - gn * p.g_h * p.g_w;
      const int gi = (int)p.w_div.div((uint32_t)rem);
      const int gj = rem - gi * p.g_w;
      const int oy = gi * p.y_step + p.y_offh;
      const int ox = gj * p.y_step + p.y_offw;
      float* yrow = p.y + ((gn * p.y_h + oy) * p.y_w + ox) * p.y_ps;
      const float* xrow = BP && bnp ? p.bx + ((gn * p.y_h + oy) * p.y_w + ox) * p.bx_ps : nullptr;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + j * 16 + r;
        if (n >= p.n) continue;
        float v = acc[i][j][e];
        if (p.bias) v += p.bias[n];
        if (p.beta != 0.f) v += p.beta * yrow[n];
        yrow[n] = v;
        if (BP && bnp) {
          const float x = xrow[n];
          const float gv = (p.brelu && !(__builtin_fmaf(x, bsc[j], bsh[j]) > 0.f)) ? 0.f : v;
          csum[j] += gv;
          csq[j] += gv * (x - bmn[j]) * bis[j];
        } else {
          csum[j] += v;
          csq[j] += v * v;
        }
      }
    }
  }
  // the VALU remainder's outputs: the 4 lane groups' K shares summed (every group then holds
  // pixel i*16 + r's sums); lane group g writes the channels q = g (mod 4)
  float rsum[NR > 0 ? NR : 1], rsq[NR > 0 ? NR : 1];
  if constexpr (NR > 0) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < NR; ++q) {
        racc[i][q] += __shfl_xor(racc[i][q], 16, 64);
        racc[i][q] += __shfl_xor(racc[i][q], 32, 64);
      }
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      rsum[q] = 0.f;
      rsq[q] = 0.f;
      if ((q & 3) != g) continue;
      const int n = n0 + BN + q;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = mw + i * 16 + r;
        const bool mok = m < M && n < p.n;
        const int mm = m < M ? m : 0;
        const int gn = (int)p.hw_div.div((uint32_t)mm);
        const int rem = mm - gn * p.g_h * p.g_w;
        const int gi = (int)p.w_div.div((uint32_t)rem);
        const int gj = rem - gi * p.g_w;
        float* yp = p.y + ((gn * p.y_h + gi * p.y_step + p.y_offh) * p.y_w + gj * p.y_step +
                           p.y_offw) * p.y_ps + n;
        float v = racc[i][q];
        if (p.bias) v += p.bias[n < p.n ? n : 0];
        if (p.beta != 0.f && mok) v += p.beta * *yp;
        if (mok) *yp = v;
        if (BP && bnp) {  // producer BatchNorm partials of remainder channel n
          const int nc = n < p.n ? n : p.n - 1;
          const __amdgpu_buffer_rsrc_t bxr = make_rsrc(p.bx, p.bx_bytes);
          const float x = load1(bxr, mok ? (uint32_t)(pix_of(mm) * p.bx_ps + n) * 4u : kOOB);
          const float gv =
              (p.brelu && !(__builtin_fmaf(x, p.bsave[2 * p.n + nc], p.bsave[3 * p.n + nc]) > 0.f))
                  ? 0.f : v;
          rsum[q] += mok ? gv : 0.f;
          rsq[q] += mok ? gv * (x - p.bsave[nc]) * p.bsave[p.n + nc] : 0.f;
        } else {
          rsum[q] += mok ? v : 0.f;
          rsq[q] += mok ? v * v : 0.f;
        }
      }
    }
  }
  if (p.stats) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      csum[j] += __shfl_xor(csum[j], 16, 64);
      csum[j] += __shfl_xor(csum[j], 32, 64);
      csq[j] += __shfl_xor(csq[j], 16, 64);
      csq[j] += __shfl_xor(csq[j], 32, 64);
    }
    if constexpr (NR > 0) {  // sum over the wave's pixels (the 16 lanes r of group g)
#pragma unroll
      for (int q = 0; q < NR; ++q) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          rsum[q] += __shfl_xor(rsum[q], o, 64);
          rsq[q] += __shfl_xor(rsq[q], o, 64);
        }
      }
      if (r == 0) {
#pragma unroll
        for (int q = 0; q < NR; ++q) {
          if ((q & 3) != g) continue;
          red[wave][0][BN + q] = rsum[q];
          red[wave][1][BN + q] = rsq[q];
        }
      }
    }
    // partial row of this workgroup: class-major over the stride-parity classes (z)
    const int rows = gridDim.x * gridDim.z;
    const int srow = blockIdx.z * gridDim.x + bm;
    if (KS > 1) {  // wave 0 holds the whole row tile
      if (g == 0) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + j * 16 + r;
          if (n >= p.n) continue;
          p.stats[srow * p.n + n] = csum[j];
          p.stats[(rows + srow) * p.n + n] = csq[j];
        }
      }
      return;
    }
    if (g == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        red[wave][0][j * 16 + r] = csum[j];
        red[wave][1][j * 16 + r] = csq[j];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < BN + NR; c += 256) {
      if (n0 + c >= p.n) continue;
      float s = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
      float s2 = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
      p.stats[srow * p.n + n0 + c] = s;
      p.stats[(rows + srow) * p.n + n0 + c] = s2;
    }
  }
}


// ----------------------------------------------------- 1x1 GEMM (persistent) ----
// Large-M 1x1 / stride-1 convs (the layer-1 64 <-> 256 expansions and the 256 -> 64
// reductions at full resolution) and their data gradients: Y[m][n] = sum_k X[m][k] W[n][k]
// with W packed [Npad][K4] (mode 0; mode 1 for the data gradient is the same form).
// The gather kernel gives each wave ONE 32-row tile with K = 64 (4 chunks): a full
// load-latency prologue and an epilogue per 256 MFMAs, weights re-read per wave
// (PMC: 52 % of wave cycles waiting, MFMA 36 % busy).  Here a workgroup stages its N block
// of W (BN x K, zero past K) in LDS once; its 4 waves then stream row tiles of 16*TM pixels
// (tile = blockIdx.x*4 + wave, + gridDim.x*4 per step) with the A fragments loaded two K
// chunks ahead ACROSS tile boundaries, so the next tile's loads are in flight during this
// tile's MFMAs and epilogue.  BN statistics accumulate over the wave's tiles: one partial
// row per workgroup.
struct Gemm1 {
  const float* a;
  int a_ps, a_c, a_c4, M;
  const float* w;       // packed rows of a_c4 floats
  int n;                // GEMM N (real)
  const float* bias;
  float* y;
  int y_ps;
  float beta;
  float* stats;         // [2][gridDim.x][n] or null
  uint32_t a_bytes, w_bytes;
  int vec;              // y 16-byte aligned with y_ps % 4 == 0 (else 4-byte stores)
  // data gradient with bx set (round 6): stats receives the producer BatchNorm's backward
  // partials (sum g, sum g*xhat; g = y masked by the ReLU recomputed from bx), as IGemm
  const float* bx;
  int bx_ps, brelu;
  const float* bsave;
  uint32_t bx_bytes;
};

template <int TM, int TN>
__global__ __launch_bounds__(256) void gemm1x1_kernel(Gemm1 p) {
  constexpr int BN = 16 * TN;
  extern __shared__ __attribute__((aligned(16))) float bsh[];  // [BN][KL]
  __shared__ float red[4][2][BN];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int n0 = blockIdx.y * BN;
  const int nch = (p.a_c4 + 15) >> 4;   // K chunks of 16
  const int KL = nch * 16 + 4;          // LDS row stride (floats): conflict-free b128 reads
  {
    const __amdgpu_buffer_rsrc_t wr = make_rsrc(p.w, p.w_bytes);
    const int q4 = nch * 4;  // quads per staged row
    for (int i = threadIdx.x; i < BN * q4; i += 256) {
      const int nn = i / q4, q = i - nn * q4;
      const bool ok = 4 * q < p.a_c4;  // (rows past the packed Npad: range check -> 0)
      const f4 v = load4(wr, ok ? (uint32_t)((n0 + nn) * p.a_c4 + 4 * q) * 4u : kOOB);
      *reinterpret_cast<f4*>(&bsh[nn * KL + 4 * q]) = v;
    }
  }
  const __amdgpu_buffer_rsrc_t ar = make_rsrc(p.a, p.a_bytes);
  const int ntiles = (p.M + 16 * TM - 1) / (16 * TM);
  const int t0 = blockIdx.x * 4 + wave, tstep = gridDim.x * 4;
  const int iters = t0 < ntiles ? (ntiles - t0 + tstep - 1) / tstep : 0;
  const int S = iters * nch;  // (tile, chunk) steps of this wave
  const bool cpad = (p.a_c & 3) != 0;
  float bv[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + j * 16 + r;
    bv[j] = (p.bias && n < p.n) ? p.bias[n] : 0.f;
  }
  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  float csum[TN], csq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) { csum[j] = 0.f; csq[j] = 0.f; }
  const bool bnp = p.bx != nullptr;
  float pmn[TN], pis[TN], psc[TN], psh[TN];  // the producer BatchNorm's coefficients
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + j * 16 + r < p.n ? n0 + j * 16 + r : p.n - 1;
    pmn[j] = bnp ? p.bsave[n] : 0.f;
    pis[j] = bnp ? p.bsave[p.n + n] : 0.f;
    psc[j] = bnp ? p.bsave[2 * p.n + n] : 0.f;
    psh[j] = bnp ? p.bsave[3 * p.n + n] : 0.f;
  }
  const __amdgpu_buffer_rsrc_t bxr = make_rsrc(p.bx, bnp ? p.bx_bytes : 0u);
  __syncthreads();  // W staged

  auto load = [&](f4* fa, int st) {
    const int it = st / nch, c = st - it * nch;
    const int t = t0 + it * tstep;
    const int q = 16 * c + 4 * g;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = t * 16 * TM + i * 16 + r;
      const bool ok = st < S && m < p.M && q < p.a_c4;
      fa[i] = load4(ar, ok ? (uint32_t)(m * p.a_ps + q) * 4u : kOOB);
    }
  };
  auto mma = [&](f4* fa, int st) {
    const int it = st / nch, c = st - it * nch;
    if (cpad && c == nch - 1) {  // channels past a_c in the last quad (a wider buffer's)
      const int q = 16 * c + 4 * g;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        fa[i][1] = q + 1 < p.a_c ? fa[i][1] : 0.f;
        fa[i][2] = q + 2 < p.a_c ? fa[i][2] : 0.f;
        fa[i][3] = q + 3 < p.a_c ? fa[i][3] : 0.f;
      }
    }
    f4 fb[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
      fb[j] = *reinterpret_cast<const f4*>(&bsh[(j * 16 + r) * KL + 16 * c + 4 * g]);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s2], fb[j][s2], acc[i][j], 0, 0, 0);
  };
  auto epi = [&](int st) {
    const int it = st / nch, c = st - it * nch;
    if (c != nch - 1) return;
    // the tile's epilogue, then a fresh accumulator.  BN partial sums in the MFMA layout
    // (lane = column r, rows 4g..4g+3; statistics only with beta = 0), then each 16x16
    // tile is transposed inside lane quads (DPP) so a lane holds 4 consecutive channels
    // of one pixel: one 16-byte store instead of four 4-byte ones.
    const int t = t0 + it * tstep;
    const int k = r & 3, qc = 4 * (r >> 2);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int mb = t * 16 * TM + i * 16 + 4 * g;
      if (p.stats && bnp) {  // producer BatchNorm partials: one batch of range-checked loads
        float xv[4][TN];
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int n = n0 + j * 16 + r;
            xv[e][j] = load1(bxr, mb + e < p.M && n < p.n
                                      ? (uint32_t)((mb + e) * p.bx_ps + n) * 4u : kOOB);
          }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const bool ok = mb + e < p.M && n0 + j * 16 + r < p.n;
            const float v = acc[i][j][e];
            const float x = xv[e][j];
            const float gv = (p.brelu && !(__builtin_fmaf(x, psc[j], psh[j]) > 0.f)) ? 0.f : v;
            csum[j] += ok ? gv : 0.f;
            csq[j] += ok ? gv * (x - pmn[j]) * pis[j] : 0.f;
          }
        }
      } else if (p.stats) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if (mb + e < p.M && n0 + j * 16 + r < p.n) {
              const float v = acc[i][j][e] + bv[j];
              csum[j] += v;
              csq[j] += v * v;
            }
          }
        }
      }
      const int m = mb + k;
      float* yrow = p.y + (int64_t)m * p.y_ps;
      f4 yold[TN];  // beta: loaded before any store (one round trip per row tile)
      if (p.beta != 0.f) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + j * 16 + qc;
          yold[j] = (p.vec && m < p.M && n + 3 < p.n) ? *reinterpret_cast<const f4*>(yrow + n)
                                                      : f4{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f4 v = acc[i][j];
        acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
        quad_transpose(v, k);
        const int n = n0 + j * 16 + qc;
        if (m >= p.M || n >= p.n) continue;
        if (p.bias) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] += n + q < p.n ? p.bias[n + q] : 0.f;
        }
        if (p.vec && n + 3 < p.n) {
          if (p.beta != 0.f) v += p.beta * yold[j];
          *reinterpret_cast<f4*>(yrow + n) = v;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (n + q < p.n) yrow[n + q] = p.beta != 0.f ? v[q] + p.beta * yrow[n + q] : v[q];
        }
      }
    }
  };
  // Two chunks' loads in flight; a tile's epilogue stores go out after the loads of the
  // next two chunks (vmcnt counts stores too: a load issued after them would wait for them)
  if (S > 0) {
    f4 fa0[TM], fa1[TM];
    load(fa0, 0);
    load(fa1, 1);
    for (int st = 0; st < S; st += 2) {
      mma(fa0, st);
      load(fa0, st + 2);
      epi(st);
      if (st + 1 < S) {
        mma(fa1, st + 1);
        load(fa1, st + 3);
        epi(st + 1);
      }
    }
  }
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
    __syncthreads();
    const int rows = gridDim.x;
    for (int c = threadIdx.x; c < BN; c += 256) {
      if (n0 + c >= p.n) continue;
      p.stats[blockIdx.x * p.n + n0 + c] = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
      p.stats[(rows + blockIdx.x) * p.n + n0 + c] =
          red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
    }
  }
}

// ------------------------------------------------------ direct 3x3 (LDS) ----
// 3x3 / stride-1 / pad-1 convolutions (the HRNet branch convs) — forward, and the
// data gradient with flipped taps and mode-1 weights.  A workgroup owns an output
// tile of (2*TM) rows x 32 columns of one image; per slab of <= 32 input channels it
// stages the (2*TM+2) x 34 halo tile in LDS once (zero halo, zero channel padding),
// then builds every tap's A fragment from LDS with one ds_read_b128 per lane.  The
// gather kernel re-reads each input element once per tap through L1/L2; here it is
// read once (+ halo).  K order inside a slab is (tap, quad), lane group g taking quad
// 4c+g of chunk c (as igemm_kernel), so B comes from the same packed weights.
struct DConv {
  const float* a;
  int a_ps, a_c, a_c4, img_h, img_w;
  int tiles_h, tiles_w;  // output tiles per image
  int cs4;               // channel quads per slab
  const float* w;        // packed [Npad][9][a_c4]
  uint32_t a_bytes, w_bytes;
  int n;
  const float* bias;
  float* y;
  int y_ps;
  float beta;
  float* stats;  // [2][gridDim.x][n] or null
  // Forward (FLIP = false): the input is the pre-BN output of a BatchNorm(+ReLU) layer
  // whose normalised activation is never stored: staging applies relu?(a*scale + shift)
  // (isave = that layer's (mean, invstd, scale, shift) [4][a_c]) to in-image pixels, the
  // zero halo stays zero.
  const float* isave;
  int irelu;
  // Data gradient (FLIP = true): this output is the gradient of such a layer's (never
  // stored) output; the epilogue writes that layer's BatchNorm backward partials (sum g,
  // sum g*xhat; g = the gradient masked by its ReLU) into stats instead of (sum, sum^2).
  // bx = the layer's pre-BN tensor (same pixels and channels as y), bsave its [4][n].
  const float* bx;
  int bx_ps, brelu;
  const float* bsave;
  uint32_t bx_bytes;  // bx extent for the range-checked epilogue loads
  int vec_out;  // y 16-byte aligned, y_ps % 4 == 0, no statistics with beta != 0
};

constexpr int kDcBW = 32;     // tile columns
constexpr int kDcMaxCs4 = 8;  // quads per slab
// (A offset, weight offset) of every K step of a slab (chunks of 4 (tap, quad) steps, an
// even number of chunks, + the 2 chunks the loop prefetches past the end), in LDS after
// the tile and the remainder weights
constexpr int kDcTab = ((9 * kDcMaxCs4 + 7) / 8) * 8 + 32;  // (+ 8 KS, KS <= 4)

// One output tile: bm = tile index (image-major), by = N block, nrows = tiles of the
// layer (rows of its BN partial statistics).
//
// NR > 0 (fp32 operands, one N block): the layer's last NR output channels (N = 16*TN +
// NR, NR in {2, 4, 8}: the 18 / 36 / 72-channel branches) are computed on the VALU
// beside the MFMAs instead of in a further 16-wide MFMA tile that would be mostly
// padding: lane = one output pixel of the wave's 16*TM (and, at TM = 2, one half of the
// NR channels), v_fma_f32 chains over the same (tap, channel) K order the chunks walk,
// with the remainder weights of the slab staged in LDS (broadcast reads).  The MFMA work
// of an 18-channel layer halves (32 -> 16 columns), of a 36-channel one drops by 1/3.
// BNX (compile time, so the plain instances carry none of it): 1 = input BatchNorm in the
// staging (DConv::isave, forward), 2 = producer BatchNorm backward partials in the
// epilogue (DConv::bx, data gradient).
// NW = waves per workgroup (4, or 8 with TM = 2: the same 8-row tile as TM = 4, each wave
// owning one row -- twice the waves per SIMD for the same LDS tile)
// KS > 1 (NW = 4 KS, NR = 0, fp32 operands): the 4 row waves' tile of the NW = 4 form with
// the K chunk pairs split between KS wave sets (set s: pairs s, s + KS, s + 2 KS, ...), sets
// 1 .. KS-1's accumulators added to set 0's through LDS in a fixed order before the epilogue
// -- KS waves per SIMD for layers whose tiles give one workgroup per CU (set_tune key 15)
template <int TM, int TN, bool FLIP, bool BF, int NR = 0, int BNX = 0, int NW = 4,
          int KS = 1>
__device__ __forceinline__ void dconv3_body(const DConv& p, const int bm, const int by,
                                            const int nrows, float* __restrict__ tile) {
  constexpr int NT = 64 * NW;
  constexpr int NWR = NW / KS;  // waves per K share: the tile's row waves
  static_assert(KS == 1 || (NW == 4 * KS && NR == 0 && !BF), "K split form");
  constexpr int BH = NWR * TM / 2, LH = BH + 2, LW = kDcBW + 2;
  constexpr int BN = 16 * TN;
  constexpr int BNT = BN + NR;             // channels of this block (MFMA + VALU)
  static_assert(NR == 0 || (!BF && NR <= 8), "remainder shape");
  __shared__ float red[NW][2][BNT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave % NWR, kp = wave / NWR;  // row wave, K share
  const int g = lane >> 4, r = lane & 15;
  const int per_img = p.tiles_h * p.tiles_w;
  const int img = bm / per_img;
  const int trem = bm - img * per_img;
  const int th = trem / p.tiles_w;
  const int oh0 = th * BH, ow0 = (trem - th * p.tiles_w) * kDcBW;
  // first output row of this wave (K shares > 0 of the KS form: past the image, so their
  // epilogue stores, loads and statistics are all masked off)
  const int ohw = kp ? (1 << 24) : oh0 + wr * (TM / 2);
  const int n0 = by * BNT;  // (NR > 0 with two N blocks: 72 = 2 x (32 + 4), set_tune key 14)
  const int kk4 = 9 * p.a_c4;
  const int csp = p.cs4 * 4 + 4;  // LDS floats per pixel (+4: bank spread)
  const int Q = p.a_c4 >> 2;

  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int trow = wr * (TM / 2) + (i >> 1), tcol = (i & 1) * 16 + r;
    abase[i] = ((trow + 1) * LW + tcol + 1) * csp;
  }
  const __amdgpu_buffer_rsrc_t arsrc = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t wrsrc = make_rsrc(p.w, p.w_bytes);
  uint32_t wrow[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) wrow[j] = (uint32_t)((n0 + j * 16 + r) * kk4) * 4u;

  f4 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const f4* fa, const f4* fb) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
  };
  // VALU remainder: lane (g, r) multiplies the A fragments it already holds (pixels
  // i*16 + r of its TM row tiles, the 4 channels of K step 4c + g) with that K step's
  // remainder weights; the 4 lane groups' shares are summed at the end.  The slab's
  // remainder weights rw[NR][(tap, quad) step][4] live in LDS.
  float* const rw = tile + LH * LW * csp;
  // floats per remainder channel in rw: the K steps of an even number of chunks (the main
  // loop runs chunks in pairs), zero past the slab's 9 x qs steps
  const int rws = ((9 * p.cs4 + 7) >> 3) * 32;
  int2* const tab = reinterpret_cast<int2*>(rw + NR * rws);
  float racc[TM][NR > 0 ? NR : 1];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) racc[i][j] = 0.f;

  const int img_base = img * p.img_h;
  for (int q0 = 0; q0 < Q; q0 += p.cs4) {
    const int qs = Q - q0 < p.cs4 ? Q - q0 : p.cs4;
    // ---- stage the halo tile of this slab (zero outside the image / past a_c) ----
    __syncthreads();
    const int nch = (9 * qs + 3) >> 2;
    {  // the slab's K-step table: entry k = (tap, quad) step k of the chunk sequence
      const int k = threadIdx.x;
      // (steps past the 9 taps: zero weights; the KS form prefetches up to 2 (KS - 1)
      //  chunks further)
      if (k < ((nch + 1) >> 1) * 8 + 8 * KS) {
        const int t = k / qs, q = k - t * qs;
        const bool tv = t < 9;
        const int tt = tv ? t : 0;
        const int dh = tt / 3 - 1, dw = tt - 3 * (tt / 3) - 1;
        const int tl = FLIP ? 8 - tt : tt;
        tab[k] = make_int2((dh * LW + dw) * csp + 4 * q,
                           tv ? (int)((uint32_t)(tl * p.a_c4 + (q0 + q) * 4) * 4u) : (int)kOOB);
      }
    }
    if constexpr (NR > 0) {  // remainder weights of the slab [j][(tap, quad)][4], FLIP
      const int per = ((9 * qs + 7) >> 3) * 32;  // whole chunk pairs: zero tail
      for (int i = threadIdx.x; i < NR * per; i += NT) {
        const int j = i / per, rem = i - j * per;
        const int t = rem / (qs * 4), c = rem - t * (qs * 4);
        const int tl = FLIP ? 8 - t : t;
        rw[j * rws + rem] =
            t < 9 ? p.w[(int64_t)(n0 + BN + j) * kk4 + tl * p.a_c4 + q0 * 4 + c] : 0.f;
      }
    }
    // thread -> (channel quad q = tid % qs, pixels pb, pb + pstride, ...); SB loads in
    // flight per thread before their LDS stores (few round trips, few extra registers)
    constexpr int SB = 3;
    {
    const int sq = threadIdx.x % qs, pb = threadIdx.x / qs, pstride = NT / qs;
    const int c = (q0 + sq) * 4;
    const bool cpad = c + 4 > p.a_c;
    // input BatchNorm (FLIP = false only): this thread's channel quad's scale / shift
    f4 isc, ish;
    if (BNX == 1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ch = c + k < p.a_c ? c + k : p.a_c - 1;
        isc[k] = p.isave[2 * p.a_c + ch];
        ish[k] = p.isave[3 * p.a_c + ch];
      }
    }
    if (pb < pstride) {
      for (int pix0 = pb; pix0 < LH * LW; pix0 += SB * pstride) {
        f4 v[SB];
        bool okv[SB];
#pragma unroll
        for (int u = 0; u < SB; ++u) {
          const int pix = pix0 + u * pstride;
          const int lr = pix / LW, lc = pix - lr * LW;
          const int ih = oh0 - 1 + lr, iw = ow0 - 1 + lc;
          const bool ok = pix < LH * LW && (unsigned)ih < (unsigned)p.img_h &&
                          (unsigned)iw < (unsigned)p.img_w;
          okv[u] = ok;
          if (VAE2_ABLATE & 1) v[u] = f4{(float)pix, (float)ih, (float)iw, (float)c};
          else
          v[u] = load4(arsrc, ok ? (uint32_t)(((img_base + ih) * p.img_w + iw) * p.a_ps + c) * 4u
                                 : kOOB);
        }
#pragma unroll
        for (int u = 0; u < SB; ++u) {
          const int pix = pix0 + u * pstride;
          if (pix >= LH * LW) break;
          if (BNX == 1 && okv[u]) {  // = bn_apply_body's arithmetic
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float t = __builtin_fmaf(v[u][k], isc[k], ish[k]);
              v[u][k] = (p.irelu && t < 0.f) ? 0.f : t;
            }
          }
          if (cpad) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (c + k >= p.a_c) v[u][k] = 0.f;
          }
          *reinterpret_cast<f4*>(&tile[pix * csp + 4 * sq]) = v[u];
        }
      }
    }
    }
    __syncthreads();
    // ---- 9 taps x qs quads of K from LDS ----
    // chunk c, lane group g: K step 4c + g, its A / weight offsets from the table
    int kc = g + 8 * kp;  // (K share kp starts at chunk pair kp)
    auto load = [&](f4* fa, f4* fb) {
      const int2 e = tab[kc];
      kc += 4;
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const f4*>(&tile[abase[i] + e.x]);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = load4(wrsrc, wrow[j] + (uint32_t)e.y);
    };
    // the remainder's share of a chunk: this lane's K step (4c + g) against the A
    // fragments of the MFMAs (steps past the 9 taps meet the zeroed tail of rw)
    int rch = 0;
    auto rem = [&](const f4* fa) {
      if constexpr (NR > 0) {
        const int ks = 4 * rch + g;
        ++rch;
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          const f4 wv = *reinterpret_cast<const f4*>(&rw[j * rws + 4 * ks]);
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            racc[i][j] = __builtin_fmaf(fa[i][0], wv[0], racc[i][j]);
            racc[i][j] = __builtin_fmaf(fa[i][1], wv[1], racc[i][j]);
            racc[i][j] = __builtin_fmaf(fa[i][2], wv[2], racc[i][j]);
            racc[i][j] = __builtin_fmaf(fa[i][3], wv[3], racc[i][j]);
          }
        }
      }
    };
    if (!BF) {
      load(fa0, fb0);
      for (int ch = 2 * kp; ch < ((VAE2_ABLATE & 4) ? 0 : nch); ch += 2 * KS) {
        load(fa1, fb1);
        if (KS > 1) kc += 8 * (KS - 1);  // (the other shares' pairs)
        mma(fa0, fb0);
        rem(fa0);
        load(fa0, fb0);
        mma(fa1, fb1);
        rem(fa1);
      }
    } else {  // bf16 operands: one 16x16x32 MFMA per chunk pair
      load(fa0, fb0);
      load(fa1, fb1);
      for (int ch = 0; ch < nch; ch += 2) {
        bf16x8 A[TM], B[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) A[i] = pack_bf16(fa0[i], fa1[i]);
#pragma unroll
        for (int j = 0; j < TN; ++j) B[j] = pack_bf16(fb0[j], fb1[j]);
        load(fa0, fb0);
        load(fa1, fb1);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], B[j], acc[i][j], 0, 0, 0);
      }
    }
  }

  if constexpr (KS > 1) {  // K shares 1 .. KS-1's accumulators onto share 0's (fixed order)
    __syncthreads();  // every wave's last reads of the tile are done
    f4* const kred = reinterpret_cast<f4*>(tile);  // [KS - 1][NWR][TM][TN][64]
    if (kp) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          kred[((((kp - 1) * NWR + wr) * TM + i) * TN + j) * 64 + lane] = acc[i][j];
    }
    __syncthreads();
    if (!kp) {
#pragma unroll
      for (int sh = 0; sh < KS - 1; ++sh)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] += kred[(((sh * NWR + wr) * TM + i) * TN + j) * 64 + lane];
    }
  }

  // ---- epilogue (bias, beta*y, BN partial statistics) ----
  float csum[TN], csq[TN];
  // producer BatchNorm backward partials (FLIP with bx): per-column mean, invstd, scale,
  // shift of that layer (= bn_bwd_reduce_body's arithmetic, element by element)
  constexpr bool bnp = BNX == 2;
  float bmn[TN], bis[TN], bsc[TN], bsh[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    csum[j] = 0.f; csq[j] = 0.f;
    if (bnp) {
      const int n = n0 + j * 16 + r < p.n ? n0 + j * 16 + r : p.n - 1;
      bmn[j] = p.bsave[n]; bis[j] = p.bsave[p.n + n];
      bsc[j] = p.bsave[2 * p.n + n]; bsh[j] = p.bsave[3 * p.n + n];
    }
  }
  if (p.vec_out) {
    // statistics in the MFMA layout (beta = 0 whenever they are requested), then each
    // 16x16 tile transposed inside lane quads: one 16-byte store per lane and tile
    const int k = r & 3, qc = 4 * (r >> 2);
    // beta (a data gradient summed onto a GradLink buffer): every old output quad of the
    // tile loaded before any store (loads cannot pass the stores to y: one round trip
    // instead of one per quad)
    constexpr bool PFA = TM * TN <= 8;
    f4 yold[PFA ? TM : 1][TN];
    auto yrow_of = [&](int i) {
      const int oh = ohw + (i >> 1), ow = ow0 + (i & 1) * 16 + g * 4 + k;
      const bool pok = oh < p.img_h && ow < p.img_w;
      return pok ? p.y + ((int64_t)(img_base + oh) * p.img_w + ow) * p.y_ps : nullptr;
    };
    auto prefetch = [&](int i, f4* yo) {
      const float* yr = yrow_of(i);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + j * 16 + qc;
        yo[j] = (yr && n + 3 < p.n) ? *reinterpret_cast<const f4*>(yr + n) : f4{0.f, 0.f, 0.f, 0.f};
      }
    };
    if (PFA && p.beta != 0.f) {
#pragma unroll
      for (int i = 0; i < (PFA ? TM : 1); ++i) prefetch(i, yold[i]);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int oh = ohw + (i >> 1);
      if (p.stats && bnp) {
        // the row tile's 4 x TN pre-BN values in one batch of range-checked loads (one
        // round trip; loads guarded by branches waited on each element in turn)
        const __amdgpu_buffer_rsrc_t bxr = make_rsrc(p.bx, p.bx_bytes);
        float xv[4][TN];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int ow = ow0 + (i & 1) * 16 + g * 4 + e;
          const bool pin = oh < p.img_h && ow < p.img_w;
          const int64_t pix = pin ? (int64_t)(img_base + oh) * p.img_w + ow : 0;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int n = n0 + j * 16 + r;
            xv[e][j] = load1(bxr, pin && n < p.n ? (uint32_t)((pix * p.bx_ps + n) * 4) : kOOB);
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int ow = ow0 + (i & 1) * 16 + g * 4 + e;
          const bool pin = oh < p.img_h && ow < p.img_w;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int n = n0 + j * 16 + r;
            const float v = acc[i][j][e] + (p.bias && n < p.n ? p.bias[n] : 0.f);
            const float x = xv[e][j];
            const float gv = (p.brelu && !(__builtin_fmaf(x, bsc[j], bsh[j]) > 0.f)) ? 0.f : v;
            const bool ok = pin && n < p.n;
            csum[j] += ok ? gv : 0.f;
            csq[j] += ok ? gv * (x - bmn[j]) * bis[j] : 0.f;
          }
        }
      } else if (p.stats) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int ow = ow0 + (i & 1) * 16 + g * 4 + e;
          if (oh >= p.img_h || ow >= p.img_w) continue;
          const int64_t pix = (int64_t)(img_base + oh) * p.img_w + ow;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int n = n0 + j * 16 + r;
            if (n >= p.n) continue;
            const float v = acc[i][j][e] + (p.bias ? p.bias[n] : 0.f);
            if (bnp) {
              const float xv = p.bx[pix * p.bx_ps + n];
              const float gv = (p.brelu && !(__builtin_fmaf(xv, bsc[j], bsh[j]) > 0.f)) ? 0.f : v;
              csum[j] += gv;
              csq[j] += gv * (xv - bmn[j]) * bis[j];
            } else {
              csum[j] += v;
              csq[j] += v * v;
            }
          }
        }
      }
      float* yrow = yrow_of(i);
      const bool pok = yrow != nullptr;
      f4 yrt[PFA ? 1 : TN];
      if (!PFA && p.beta != 0.f) prefetch(i, yrt);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f4 v = acc[i][j];
        quad_transpose(v, k);
        const int n = n0 + j * 16 + qc;
        if (!pok || n >= p.n) continue;
        if (p.bias) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] += n + q < p.n ? p.bias[n + q] : 0.f;
        }
        if (n + 3 < p.n) {
          if (p.beta != 0.f) v += p.beta * (PFA ? yold[PFA ? i : 0][j] : yrt[PFA ? 0 : j]);
          if (!(VAE2_ABLATE & 2) || v[0] == 1234.5f) *reinterpret_cast<f4*>(yrow + n) = v;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (n + q < p.n) yrow[n + q] = p.beta != 0.f ? v[q] + p.beta * yrow[n + q] : v[q];
        }
      }
    }
  } else
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int oh = ohw + (i >> 1);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ow = ow0 + (i & 1) * 16 + g * 4 + e;
      if (oh >= p.img_h || ow >= p.img_w) continue;
      const int64_t pix = (int64_t)(img_base + oh) * p.img_w + ow;
      float* yrow = p.y + pix * p.y_ps;
      const float* xrow = bnp ? p.bx + pix * p.bx_ps : nullptr;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + j * 16 + r;
        if (n >= p.n) continue;
        float v = acc[i][j][e];
        if (p.bias) v += p.bias[n];
        if (p.beta != 0.f) v += p.beta * yrow[n];
        if (!(VAE2_ABLATE & 2) || v == 1234.5f) yrow[n] = v;
        if (bnp) {
          const float xv = xrow[n];
          const float gv = (p.brelu && !(__builtin_fmaf(xv, bsc[j], bsh[j]) > 0.f)) ? 0.f : v;
          csum[j] += gv;
          csq[j] += gv * (xv - bmn[j]) * bis[j];
        } else {
          csum[j] += v;
          csq[j] += v * v;
        }
      }
    }
  }
  // the VALU remainder's outputs: the 4 lane groups' K-step shares summed (every group
  // then holds pixel i*16 + r's sums); lane group g writes the channels j = g (mod 4)
  float rsum[NR > 0 ? NR : 1], rsq[NR > 0 ? NR : 1];
  if constexpr (NR > 0) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        racc[i][j] += __shfl_xor(racc[i][j], 16, 64);
        racc[i][j] += __shfl_xor(racc[i][j], 32, 64);
      }
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      rsum[j] = 0.f;
      rsq[j] = 0.f;
      if ((j & 3) != g) continue;
      const int n = n0 + BN + j;
      float bxv[TM];  // the pre-BN values of the TM pixels, one batch of loads (bnp)
      if (bnp) {
        const __amdgpu_buffer_rsrc_t bxr = make_rsrc(p.bx, p.bx_bytes);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int oh = ohw + (i >> 1), ow = ow0 + (i & 1) * 16 + r;
          const bool in = oh < p.img_h && ow < p.img_w;
          const int64_t pix = (int64_t)(img_base + (in ? oh : 0)) * p.img_w + (in ? ow : 0);
          bxv[i] = load1(bxr, in ? (uint32_t)((pix * p.bx_ps + n) * 4) : kOOB);
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int oh = ohw + (i >> 1), ow = ow0 + (i & 1) * 16 + r;
        const bool in = oh < p.img_h && ow < p.img_w;
        const int64_t pix = (int64_t)(img_base + (in ? oh : 0)) * p.img_w + (in ? ow : 0);
        float* yp = p.y + pix * p.y_ps + n;
        float v = racc[i][j];
        if (p.bias) v += p.bias[n];
        if (p.beta != 0.f && in) v += p.beta * *yp;
        if (in && (!(VAE2_ABLATE & 2) || v == 1234.5f)) *yp = v;
        if (bnp) {
          const float xv = bxv[i];
          const float gv = (p.brelu && !(__builtin_fmaf(xv, p.bsave[2 * p.n + n],
                                                        p.bsave[3 * p.n + n]) > 0.f)) ? 0.f : v;
          rsum[j] += in ? gv : 0.f;
          rsq[j] += in ? gv * (xv - p.bsave[n]) * p.bsave[p.n + n] : 0.f;
        } else {
          rsum[j] += in ? v : 0.f;
          rsq[j] += in ? v * v : 0.f;
        }
      }
    }
  }
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
    if constexpr (NR > 0) {  // sum over the wave's pixels (the 16 lanes r of group g)
#pragma unroll
      for (int j = 0; j < NR; ++j) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          rsum[j] += __shfl_xor(rsum[j], o, 64);
          rsq[j] += __shfl_xor(rsq[j], o, 64);
        }
      }
      if (r == 0) {
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          if ((j & 3) != g) continue;
          red[wave][0][BN + j] = rsum[j];
          red[wave][1][BN + j] = rsq[j];
        }
      }
    }
    __syncthreads();
    const int rows = nrows;
    for (int c = threadIdx.x; c < BNT; c += NT) {
      if (n0 + c >= p.n) continue;
      float s = red[0][0][c], s2 = red[0][1][c];
#pragma unroll
      for (int w = 1; w < NW; ++w) {
        s += red[w][0][c];
        s2 += red[w][1][c];
      }
      p.stats[bm * p.n + n0 + c] = s;
      p.stats[(rows + bm) * p.n + n0 + c] = s2;
    }
  }
}

template <int TM, int TN, bool FLIP, bool BF = false, int NR = 0, int BNX = 0, int NW = 4,
          int KS = 1>
__global__ __launch_bounds__(64 * NW, (TM == 4 && TN == 4 && NR == 0 && NW == 4) ? 3 : 1) void dconv3_kernel(DConv p) {
  static_assert(BNX == 0 || (!BF && (BNX == 1) != FLIP), "input BN: forward; partials: dgrad");
  extern __shared__ __attribute__((aligned(16))) float tile[];
  dconv3_body<TM, TN, FLIP, BF, NR, BNX, NW, KS>(p, xcd_remap(blockIdx.x, gridDim.x),
                                                 blockIdx.y, gridDim.x, tile);
}

// Up to kDcGroup independent layers with the same tile shape in one launch (the lock-
// stepped HRNet branches of one depth level: the low-resolution ones alone leave most
// of the chip idle).  The 1-D grid is the concatenation of each layer's (tiles x N
// blocks); the XCD remap runs over the whole grid, then the block finds its layer.
constexpr int kDcGroup = 4;
struct DConvGroup {
  DConv p[kDcGroup];
  int start[kDcGroup + 1];
  int tiles[kDcGroup];
  int n;
};

template <int TM, int TN, bool FLIP, bool BF = false>
__global__ __launch_bounds__(256) void dconv3_group_kernel(DConvGroup gp) {
  extern __shared__ __attribute__((aligned(16))) float tile[];
  const int idx = xcd_remap(blockIdx.x, gridDim.x);
  int j = 0;
#pragma unroll
  for (int k = 1; k < kDcGroup; ++k) j += (k < gp.n && idx >= gp.start[k]) ? 1 : 0;
  const DConv p = j == 0 ? gp.p[0] : j == 1 ? gp.p[1] : j == 2 ? gp.p[2] : gp.p[3];
  const int t = j == 0 ? gp.tiles[0] : j == 1 ? gp.tiles[1] : j == 2 ? gp.tiles[2] : gp.tiles[3];
  const int st = j == 0 ? gp.start[0] : j == 1 ? gp.start[1] : j == 2 ? gp.start[2] : gp.start[3];
  const int local = idx - st;
  const int by = local / t;
  dconv3_body<TM, TN, FLIP, BF>(p, local - by * t, by, t, tile);
}

// ------------------------------------------------------------ tiling ----
struct Tile {
  int tm, tn, nblk;
  int ks = 1;  // in-workgroup K split (igemm_kernel KS)
  int nr = 0;  // output channels on the VALU beside the MFMA columns (igemm_kernel NR)
};

// Rows per workgroup and the K split: layers whose row tiles would leave the chip with
// fewer than ~2 waves per SIMD split K over the workgroup's 4 waves instead (when K has
// at least 16 chunks of 16), giving 4x the workgroups.
static int64_t igemm_rows_per_block(const Tile& t) { return (t.ks > 1 ? 16 : 64) * t.tm; }

#if VAE2_PART(0)
int g_wide_tiles = 1;
int g_ksplit = 1;    // vae2_conv2d_set_algo bit 8 disables the K split (A/B tests)
int g_bf16 = 0;      // vae2_conv2d_set_mfma_bf16: bf16 MFMA operands (fp32 accumulate)
int g_conv_algo = 0; // 0 auto, 1 gather kernel only, 2 direct wherever legal
int g_dconv_nr = 1;  // vae2_conv2d_set_algo: bit 16 clear enables the VALU remainder
int g_gemm1 = 1;     // vae2_conv2d_set_algo: bit 32 clear enables the persistent 1x1 GEMM
int g_vec_out = 1;   // vae2_conv2d_set_algo: bit 64 clear enables the quad-transposed stores
int g_dconv_nr_wide = 1;  // vae2_conv2d_set_algo: bit 128 clear enables the 32 + 4 / 64 + 8 forms
int g_igemm_minblk = 512;  // vae2_conv2d_set_tune key 0: igemm row tiles shrink to reach this grid
                           // (512 since round 6: step 909.3-910.7 -> 915.4-915.8 frames/s over 3
                           //  interleaved reps, 768: level; scripts/gpu_r6_q.sh)
// (keys 1 and 3 on by default: round-4 A/B on one box, 20-step benches twice interleaved:
//  default 820.7 / 822.4 frames/s, key 1 824.2 / 823.1, key 3 828.3 / 828.3; key 2 (8-wave
//  direct 3x3) 825.1 / 823.8 and key 0 = 1024 819.7 / 818.4 stay off)
int g_wgrad_cols = 1;     // vae2_conv2d_set_tune key 1: weight-gradient column blocks (pick_wtile)
int g_dconv_nw8 = 0;      // vae2_conv2d_set_tune key 2: direct 3x3 8-row tiles as 8 waves
int g_wgrad_nw8 = 1;      // vae2_conv2d_set_tune key 3: 3x3 weight gradients over 8 waves
// key 4: the 1x1 GEMM's N tiles per workgroup (3..8).  4 by default: the TN = 8 instance
// holds 264 VGPRs (1 wave / SIMD) and its persistent grid was sized for 3 per CU, i.e. ran in
// 3 rounds; with the grid from the occupancy query, conv_bench 64->256 forward 172 (TN 8,
// LDS-sized grid) -> 157 (TN 8) -> 131 us (TN 4, 152 VGPRs), 256->64 data gradient
// 153 -> 127 us; step 845.1 / 845.4 (8) vs 847.3 / 848.0 frames/s (4), same box.
int g_gemm1_tn = 4;
int g_gemm1_tm = 2;       // vae2_conv2d_set_tune key 5: 1x1 GEMM row tiles of 16 * TM pixels (1, 2)
int g_igemm_nr = 2;       // vae2_conv2d_set_tune key 6: igemm VALU remainder for N = 18 / 36 (1),
                          // N = 18 only (2, default: step 895.7 -> 899.8 frames/s, 3 A/B pairs)
int g_wgrad_narrow = 3;   // vae2_conv2d_set_tune key 7: wgrad_narrow.hip for 18 / 36 / 72 channels
                          // (0 off, 1 on, 2 on with register prefetch, 3 on with 8 waves:
                          //  18 / 36 / 72 ch 35.0 / 31.7 / 32.1 -> 33.0 / 31.4 / 31.2 us)
int g_igemm_tab = 1;      // vae2_conv2d_set_tune key 12: the gather GEMM's K-step table
int g_dconv_n16 = 0;      // vae2_conv2d_set_tune key 13: direct 3x3 16-channel N blocks when short of workgroups
int g_dconv_split72 = 0;  // vae2_conv2d_set_tune key 14: 72-channel direct 3x3 as two 32 + 4 N blocks
int g_dconv_ksp = 1;      // vae2_conv2d_set_tune key 15: direct 3x3 K split when short of workgroups (0 off, 1: 2 shares / 8 waves, 2: 4 shares / 16 waves)
int g_wgrad_wgs = 1024;   // vae2_conv2d_set_tune key 18: gather weight-gradient target workgroups
extern int g_bn_v2;       // bn.hip; vae2_conv2d_set_tune key 8
#else
extern int g_wide_tiles, g_ksplit, g_bf16, g_conv_algo, g_dconv_nr, g_gemm1, g_vec_out,
    g_dconv_nr_wide, g_igemm_minblk, g_wgrad_cols, g_dconv_nw8, g_wgrad_nw8, g_gemm1_tn,
    g_gemm1_tm, g_igemm_nr, g_wgrad_narrow, g_igemm_tab, g_dconv_n16, g_dconv_split72,
    g_dconv_ksp, g_wgrad_wgs;
#endif

// 1x1 convs with many output channels ("wide"): up to 9 column tiles per wave and
// 32 rows, so the activation rows are re-read by 2 column blocks instead of 5.
static bool wide_ok(int64_t M, int N, int taps) {
  return g_wide_tiles && taps == 1 && N > 64 && M >= 65536;
}

static Tile pick_tile(int64_t M, int N, bool wide = false) {
  Tile t;
  int tiles = (N + 15) / 16;
  if (wide && tiles > 4) {
    t.nblk = (tiles + 8) / 9;
    t.tn = (tiles + t.nblk - 1) / t.nblk;
    t.tm = 2;
    return t;
  }
  if (tiles <= 4) {
    t.tn = tiles;
    t.nblk = 1;
  } else {
    t.nblk = (tiles + 3) / 4;
    t.tn = (tiles + t.nblk - 1) / t.nblk;
  }
  // 4 waves per block, 16*TM rows per wave; large TM once there are enough rows
  t.tm = (M >= 64 * 4 * 256) ? 4 : (M >= 32 * 4 * 128 ? 2 : 1);
  return t;
}


static Tile pick_igemm_tile(int64_t M, int N, int taps, int k4, int ncls) {
  const bool wide = wide_ok(M, N, taps);
  Tile t = pick_tile(M, N, wide);
  // smaller row tiles until the grid reaches g_igemm_minblk workgroups (more waves per
  // SIMD for layers whose 4-row-tile grid leaves one wave per SIMD)
  while (!wide && g_igemm_minblk > 0 && t.tm > 1 &&
         ceil_div(M, 64 * t.tm) * t.nblk * ncls < g_igemm_minblk)
    t.tm >>= 1;
  const int64_t blocks = ceil_div(M, 64 * t.tm) * t.nblk * ncls;
  const int chunks = (taps * k4 + 15) / 16;
  if (g_ksplit && !wide && blocks < 512 && chunks >= 16) t.ks = 4;
  // tune key 6: 18 / 36 output channels as 16 + 2 / 32 + 4 (VALU remainder, fp32, no K split);
  // 2: 18 channels only
  if (g_igemm_nr && !g_bf16 && t.ks == 1 && !wide && (N == 18 || (N == 36 && g_igemm_nr == 1))) {
    t.tn = N == 18 ? 1 : 2;
    t.nr = N == 18 ? 2 : 4;
    t.nblk = 1;
  }
  return t;
}

static bool vec_ok(const float* a, int ps) {
  return ((uintptr_t)a % 16 == 0) && (ps % 4 == 0);
}


// ---------------------------------------------------- 1x1 GEMM: host dispatch ----
struct G1Tile {
  int tm = 2, tn, nblk, grid_x;
  size_t lds;
};
int gemm1_blocks_per_cu(int tm, int tn, size_t lds);

static bool gemm1_pick(const vae2_act* ad, const vae2_act* yd, int k, int stride, int pad,
                       const float* a, G1Tile* out) {
  if (!g_gemm1 || g_bf16 || g_conv_algo == 1) return false;
  if (k != 1 || stride != 1 || pad != 0 || ad->h != yd->h || ad->w != yd->w) return false;
  const int64_t M = act_pixels(yd);
  const int N = (int)yd->c;
  if (M < 65536 || N < 48 || !vec_ok(a, (int)ad->ps)) return false;
  const int k4 = round_up((int)ad->c, 4);
  const int tiles = (N + 15) / 16;
  G1Tile t;
  const int tn_max = g_gemm1_tn >= 3 && g_gemm1_tn <= 8 ? g_gemm1_tn : 4;
  t.nblk = (tiles + tn_max - 1) / tn_max;
  t.tn = (tiles + t.nblk - 1) / t.nblk;
  if (t.tn < 3) t.tn = 3;
  const int nch = (k4 + 15) / 16;
  t.lds = (size_t)16 * t.tn * (nch * 16 + 4) * sizeof(float);
  if (t.lds > 96 * 1024) return false;
  // resident workgroups per CU (registers and LDS; the TN = 8 instance holds 264 VGPRs:
  // one wave per SIMD) -- the persistent grid is exactly that many per CU
  t.tm = g_gemm1_tm == 1 ? 1 : 2;  // tune key 5: 16-row tiles (half the accumulators)
  const int per_cu = gemm1_blocks_per_cu(t.tm, t.tn, t.lds);
  const int64_t ntiles = ceil_div(M, 16 * t.tm);
  int64_t gx = 256 * per_cu / t.nblk;
  if (gx > ceil_div(ntiles, 4)) gx = ceil_div(ntiles, 4);
  t.grid_x = (int)(gx < 1 ? 1 : gx);
  if (out) *out = t;
  return true;
}

int launch_igemm(IGemm& p, int role, hipStream_t s, const char* fn, int ncls = 1);
int launch_gemm1(const float* a, const vae2_act* ad, const float* wp, uint32_t w_bytes,
                 const float* bias, float* y, const vae2_act* yd, float beta, float* stats,
                 const G1Tile& t, hipStream_t s, const char* fn, const float* bx = nullptr,
                 int bx_ps = 0, int brelu = 0, const float* bsave = nullptr,
                 uint32_t bx_bytes = 0);


#if VAE2_PART(1)
template <int TM, bool VEC, int ROLE, int KS = 1>
static void launch_tn(const IGemm& p, int tn, dim3 grid, hipStream_t s) {
  switch (tn) {
#define CASE(T) \
  case T:                                                                         \
    if (g_bf16) VAE2_LAUNCH((igemm_kernel<TM, T, VEC, ROLE, KS, true>), grid, dim3(256), 0, s, p); \
    else VAE2_LAUNCH((igemm_kernel<TM, T, VEC, ROLE, KS>), grid, dim3(256), 0, s, p);   \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4)
#undef CASE
  }
}

template <bool VEC, int ROLE>
static void launch_wide(const IGemm& p, int tn, dim3 grid, hipStream_t s) {
  switch (tn) {
#define CASE(T) \
  case T:                                                                         \
    if (g_bf16) VAE2_LAUNCH((igemm_kernel<2, T, VEC, ROLE, 1, true>), grid, dim3(256), 0, s, p); \
    else VAE2_LAUNCH((igemm_kernel<2, T, VEC, ROLE>), grid, dim3(256), 0, s, p);       \
    break;
    CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9)
#undef CASE
  }
}

template <bool VEC, int ROLE>
static void launch_nr(const IGemm& p, const Tile& t, dim3 grid, hipStream_t s) {
#define NRL(TM_)                                                                             \
  if (t.nr == 2) VAE2_LAUNCH((igemm_kernel<TM_, 1, VEC, ROLE, 1, false, 2>), grid, dim3(256), 0, s, p); \
  else VAE2_LAUNCH((igemm_kernel<TM_, 2, VEC, ROLE, 1, false, 4>), grid, dim3(256), 0, s, p);
  if (t.tm == 4) { NRL(4) }
  else if (t.tm == 2) { NRL(2) }
  else { NRL(1) }
#undef NRL
}
template <bool VEC, int ROLE>
static void launch_tm(const IGemm& p, const Tile& t, dim3 grid, hipStream_t s) {
  if (t.nr) {
    launch_nr<VEC, ROLE>(p, t, grid, s);
    return;
  }
  if (t.ks > 1) {  // (never with wide tiles: those need >= 65536 rows)
    if (t.tm == 4) launch_tn<4, VEC, ROLE, 4>(p, t.tn, grid, s);
    else if (t.tm == 2) launch_tn<2, VEC, ROLE, 4>(p, t.tn, grid, s);
    else launch_tn<1, VEC, ROLE, 4>(p, t.tn, grid, s);
    return;
  }
  if (t.tm == 2 && t.tn > 4) launch_wide<VEC, ROLE>(p, t.tn, grid, s);
  else if (t.tm == 4) launch_tn<4, VEC, ROLE>(p, t.tn, grid, s);
  else if (t.tm == 2) launch_tn<2, VEC, ROLE>(p, t.tn, grid, s);
  else launch_tn<1, VEC, ROLE>(p, t.tn, grid, s);
}

// ncls > 1: p.cls[0..ncls) hold the parity classes; the grid covers the largest one.
int launch_igemm(IGemm& p, int role, hipStream_t s, const char* fn, int ncls) {
  p.ktab = g_igemm_tab;
  int64_t M = (int64_t)p.g_n * p.g_h * p.g_w;
  if (ncls > 1) {
    M = 0;
    for (int c = 0; c < ncls; ++c) {
      IGemm::Cls& k = p.cls[c];
      k.hw_div = FastDiv((uint32_t)(k.g_h * k.g_w));
      k.w_div = FastDiv((uint32_t)k.g_w);
      const int64_t mc = (int64_t)p.g_n * k.g_h * k.g_w;
      if (mc > M) M = mc;
    }
  }
  if (M == 0) return 0;
  int max_taps = p.nth * p.ntw;
  for (int c = 0; c < ncls && ncls > 1; ++c)
    if (p.cls[c].nth * p.cls[c].ntw > max_taps) max_taps = p.cls[c].nth * p.cls[c].ntw;
  Tile t = pick_igemm_tile(M, p.n, max_taps, p.a_c4, ncls);
  p.vec_out = g_vec_out && vec_ok(p.y, p.y_ps) && !(p.stats && p.beta != 0.f);
  p.hw_div = FastDiv((uint32_t)(p.g_h * p.g_w));
  p.w_div = FastDiv((uint32_t)p.g_w);
  dim3 grid((unsigned)ceil_div(M, igemm_rows_per_block(t)), (unsigned)t.nblk, (unsigned)ncls);
  bool vec = vec_ok(p.a, p.a_ps);
  if (role == 0) {
    if (vec) launch_tm<true, 0>(p, t, grid, s);
    else launch_tm<false, 0>(p, t, grid, s);
  } else {
    if (vec) launch_tm<true, 1>(p, t, grid, s);
    else launch_tm<false, 1>(p, t, grid, s);
  }
  return check_launch(fn);
}


#endif  // VAE2_PART(1)

static int64_t igemm_rows(int64_t M, int N, int taps, int k4) {
  Tile t = pick_igemm_tile(M, N, taps, k4, 1);
  return ceil_div(M, igemm_rows_per_block(t));
}

// ------------------------------------------------------------ wgrad ----
// dW[co][(tap, ci4)] = sum_p dY[p][co] * X[src(p, tap)][ci].  MFMA m = co, n = column,
// k = pixel: lane group g takes pixels 4g..4g+3 of each 16-pixel chunk.
// Workgroup = 4 waves sharing one (co, column) tile; wave w takes chunks w, w+4, ...
// of the workgroup's pixel range, the 4 partial tiles are summed in LDS (fixed
// order) and written as one fp32 slab part[split][cout][ncol4].
struct WGrad {
  const float* x;
  int x_ps, cin, cin4, x_h, x_w;
  const float* dy;
  int dy_ps, cout, o_n, o_h, o_w;
  int k, stride, pad;
  int P, px_split;
  uint32_t x_bytes, dy_bytes;
  float* part;
  FastDiv ohw_div, ow_div, cin4_div;
};

// V4 (16-byte aligned NHWC operands): lane (g, 4Q + k) loads ONE 16-byte channel quad
// of pixel 4g + k per operand tile -- dY[px][co 4Q..4Q+3], X[src(px)][ci 4Q..4Q+3] -- and
// a 4x4 transpose inside its lane quad (quad_transpose, DPP) turns those into the MFMA
// fragments (4 pixels of one co / ci), instead of four 4-byte loads with four pixel
// address computations per operand tile.
template <int TM, int TN, bool BF = false, bool V4 = false>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(WGrad p) {
  extern __shared__ __attribute__((aligned(16))) float wred[];  // [3][TM*TN*4][64]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int ncol4 = p.k * p.k * p.cin4;
  const int co0 = blockIdx.y * 16 * TM;
  const int col0 = blockIdx.x * 16 * TN;
  const int pbeg = blockIdx.z * p.px_split;
  const int pend = min(pbeg + p.px_split, p.P);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const __amdgpu_buffer_rsrc_t dr = make_rsrc(p.dy, p.dy_bytes);

  int aco[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int co = co0 + i * 16 + r;
    aco[i] = co < p.cout ? co : -1;
  }
  int bkh[TN], bkw[TN], boff[TN];
  bool bok[TN];
  const int kq = r & 3;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col0 + j * 16 + (V4 ? 4 * (r >> 2) : r);  // (V4: the lane's channel quad)
    const int t = (int)p.cin4_div.div((uint32_t)col);
    const int ci = col - t * p.cin4;
    bkh[j] = t / p.k;
    bkw[j] = t - bkh[j] * p.k;
    bok[j] = col < ncol4 && ci < p.cin;
    boff[j] = (bkh[j] * p.x_w + bkw[j]) * p.x_ps + ci;
  }
  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const int ohw = p.o_h * p.o_w;
  // chunk loads (pixels past pend load 0), double-buffered in registers: the next
  // chunk's loads are in flight across this chunk's MFMAs
  auto load = [&](int pc, f4* fa, f4* fb) {
    if constexpr (V4) {
      const int pix = pc + 4 * g + kq;
      const bool pv = pix < pend;
      const int pp = pv ? pix : pbeg;
      const int n = (int)p.ohw_div.div((uint32_t)pp);
      const int rem = pp - n * ohw;
      const int oh = (int)p.ow_div.div((uint32_t)rem);
      const int ow = rem - oh * p.o_w;
      const uint32_t drow = (uint32_t)(pp * p.dy_ps);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int co = co0 + i * 16 + 4 * (r >> 2);
        fa[i] = load4(dr, (pv && co < p.cout) ? (drow + co) * 4u : kOOB);
      }
      const int ih0 = oh * p.stride - p.pad, iw0 = ow * p.stride - p.pad;
      const int xc = ((n * p.x_h + ih0) * p.x_w + iw0) * p.x_ps;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int ih = ih0 + bkh[j], iw = iw0 + bkw[j];
        const bool ok = pv && bok[j] && (unsigned)ih < (unsigned)p.x_h &&
                        (unsigned)iw < (unsigned)p.x_w;
        fb[j] = load4(xr, ok ? (uint32_t)(xc + boff[j]) * 4u : kOOB);
      }
      return;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int pix = pc + 4 * g + s;
      const bool pv = pix < pend;
      const int pp = pv ? pix : pbeg;
      const int n = (int)p.ohw_div.div((uint32_t)pp);
      const int rem = pp - n * ohw;
      const int oh = (int)p.ow_div.div((uint32_t)rem);
      const int ow = rem - oh * p.o_w;
      const uint32_t drow = (uint32_t)(pp * p.dy_ps);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i][s] = load1(dr, (pv && aco[i] >= 0) ? (drow + aco[i]) * 4u : kOOB);
      const int ih0 = oh * p.stride - p.pad, iw0 = ow * p.stride - p.pad;
      const int xc = ((n * p.x_h + ih0) * p.x_w + iw0) * p.x_ps;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int ih = ih0 + bkh[j], iw = iw0 + bkw[j];
        const bool ok = pv && bok[j] && (unsigned)ih < (unsigned)p.x_h &&
                        (unsigned)iw < (unsigned)p.x_w;
        fb[j][s] = load1(xr, ok ? (uint32_t)(xc + boff[j]) * 4u : kOOB);
      }
    }
  };
  auto quads = [&](f4* fa, f4* fb) {  // V4: quad loads -> fragments (after they landed)
    if constexpr (V4) {
#pragma unroll
      for (int i = 0; i < TM; ++i) quad_transpose(fa[i], kq);
#pragma unroll
      for (int j = 0; j < TN; ++j) quad_transpose(fb[j], kq);
    }
  };
  auto mma = [&](f4* fa, f4* fb) {
    quads(fa, fb);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
  };
  {
    f4 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
    int pc = pbeg + 16 * wave;
    if (!BF) {
      if (pc < pend) load(pc, fa0, fb0);
      for (; pc < pend; pc += 128) {
        load(pc + 64, fa1, fb1);
        mma(fa0, fb0);
        load(pc + 128, fa0, fb0);
        mma(fa1, fb1);
      }
    } else if (pc < pend) {  // bf16 operands: one 16x16x32 MFMA per chunk pair
      load(pc, fa0, fb0);
      load(pc + 64, fa1, fb1);
      for (; pc < pend; pc += 128) {
        bf16x8 A[TM], B[TN];
        quads(fa0, fb0);
        quads(fa1, fb1);
#pragma unroll
        for (int i = 0; i < TM; ++i) A[i] = pack_bf16(fa0[i], fa1[i]);
#pragma unroll
        for (int j = 0; j < TN; ++j) B[j] = pack_bf16(fb0[j], fb1[j]);
        load(pc + 128, fa0, fb0);
        load(pc + 192, fa1, fb1);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], B[j], acc[i][j], 0, 0, 0);
      }
    }
  }

  // cross-wave reduction in a fixed order: waves 1..3 park their tiles in LDS
  constexpr int NV = TM * TN * 4;
  if (wave > 0) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          wred[((wave - 1) * NV + (i * TN + j) * 4 + e) * 64 + lane] = acc[i][j][e];
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int w = 0; w < 3; ++w)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[i][j][e] += wred[(w * NV + (i * TN + j) * 4 + e) * 64 + lane];

  float* out = p.part + (int64_t)blockIdx.z * p.cout * ncol4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int co = co0 + i * 16 + g * 4 + e;
      if (co >= p.cout) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = col0 + j * 16 + r;
        if (col < ncol4) out[(int64_t)co * ncol4 + col] = acc[i][j][e];
      }
    }
}

// --------------------------------------------------- direct 3x3 wgrad (LDS) ----
// dW of 3x3 / stride-1 / pad-1 convs.  A workgroup owns a (co slab, ci slab) of dW
// and a run of BH x 32 pixel tiles; per tile it stages dY (transposed: [co][px]) and
// the X halo tile (transposed: [ci][halo px]) in LDS once, then every wave sweeps all
// the tile's pixels (MFMA k) for its own TN column tiles (columns = (tap, ci) of the
// slab), so no cross-wave reduction is needed.  Partial slabs part[split][co][(t,ci)]
// are summed by wgrad_reduce_kernel in a fixed order (deterministic).
struct WGrad3 {
  const float* x;
  int x_ps, cin, cin4, h, w;
  const float* dy;
  int dy_ps, cout;
  int tiles_h, tiles_w, ntiles, tiles_per_split;
  int csw, n_ci_slabs;  // channels per ci slab (multiple of 4), slabs
  uint32_t x_bytes, dy_bytes;
  float* part;  // [splits][cout][9*cin4]
  // x is the pre-BN output of a BatchNorm(+ReLU) layer whose normalised activation is
  // never stored (DConv::isave): staging applies relu?(x*scale + shift) to in-image pixels
  const float* isave;
  int irelu;
};

// NR > 0 (fp32 operands, one co slab): cout = 16*TM + NR (the 18 / 36-channel layers)
// -- the last NR output channels are computed on the VALU beside the MFMAs instead of in a
// further 16-row MFMA tile that would be mostly padding: every lane already holds the X
// fragment of its column for 4 pixels (the MFMA B operand), so it adds those pixels'
// dY[co][px] * X products for each remainder co (dY rows staged with the others) and
// the 4 lane groups' sums are combined at the end.  The MFMA work of an 18-channel
// layer halves (32 -> 16 rows), of a 36-channel one drops by 1/3.  With several co slabs
// (72 = 2 x (32 + 4)) each slab is 16*TM + NR channels wide.
// NW = waves per workgroup: 4, or 8 (each wave half the column tiles: twice the waves per
// SIMD for layers whose grid leaves one workgroup per CU)
template <int TM, int TN, int BH, bool PF, int KS, bool BF = false, int NR = 0, int NW = 4>
__global__ __launch_bounds__(64 * NW) void wgrad3_kernel(WGrad3 p) {
  constexpr int NT = 64 * NW;
  constexpr int HALO = KS / 2, TAPS = KS * KS;
  constexpr int LH = BH + KS - 1, LW = 32 + KS - 1, NPX = BH * 32, LPX = LH * LW;
  constexpr int QMAX = KS == 1 ? 16 : 9;  // channel quads per slab
  constexpr int DYS = NPX + 4;  // dY^T row stride (floats)
  constexpr int NRQ = (NR + 3) / 4;        // remainder co quads staged
  constexpr int NQ = 4 * TM + NRQ;         // dY co quads staged per tile
  static_assert(NR == 0 || (!BF && NR <= 4), "remainder shape");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* dyt = sm;                  // [16*TM + 4*NRQ][DYS]
  float* xt = sm + NQ * 4 * DYS;    // [csw + 1][LPX], row csw = zeros
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int cis = blockIdx.y % p.n_ci_slabs, cos = blockIdx.y / p.n_ci_slabs;
  const int co0 = cos * (16 * TM + NR), c0 = cis * p.csw;
  const int csw_real = p.cin4 - c0 < p.csw ? p.cin4 - c0 : p.csw;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const __amdgpu_buffer_rsrc_t dr = make_rsrc(p.dy, p.dy_bytes);

  int bbase[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = (wave * TN + j) * 16 + r;
    const int t = n / p.csw;
    const int cl = n - t * p.csw;
    const bool ok = t < TAPS && cl < csw_real;
    bbase[j] = ok ? cl * LPX + (t / KS) * LW + (t % KS) : p.csw * LPX;
  }
  for (int i = threadIdx.x; i < LPX; i += NT) xt[p.csw * LPX + i] = 0.f;
  // input BatchNorm: the slab's scale / shift (read after the tile loop's first barrier)
  __shared__ float ibn[2][QMAX * 4];
  if (p.isave && threadIdx.x < QMAX * 4) {
    const int ch = c0 + (int)threadIdx.x < p.cin ? c0 + (int)threadIdx.x : p.cin - 1;
    ibn[0][threadIdx.x] = p.isave[2 * p.cin + ch];
    ibn[1][threadIdx.x] = p.isave[3 * p.cin + ch];
  }
  auto ibn_apply = [&](f4& v, int q) {  // = bn_apply_body's arithmetic
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float t = __builtin_fmaf(v[k], ibn[0][4 * q + k], ibn[1][4 * q + k]);
      v[k] = (p.irelu && t < 0.f) ? 0.f : t;
    }
  };

  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  float racc[TN][NR > 0 ? NR : 1];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int q = 0; q < NR; ++q) racc[j][q] = 0.f;

  const int per_img = p.tiles_h * p.tiles_w;
  const int tb = blockIdx.x * p.tiles_per_split;
  const int te = tb + p.tiles_per_split < p.ntiles ? tb + p.tiles_per_split : p.ntiles;
  // Register prefetch: tile t+1's global loads are in flight while tile t computes.
  constexpr int NDY = NPX * NQ;                 // dY items (f4 = 4 co of one pixel)
  constexpr int NI = (NDY + NT - 1) / NT;         // dY items per thread
  constexpr int NX = (LPX * QMAX + NT - 1) / NT;  // X items per thread
  const int xtotal = LPX * (csw_real >> 2);
  f4 pdy[NI], pxx[NX];
  static_assert(NX <= 32, "x item mask");
  uint32_t xok = 0;  // in-image x items of the prefetched tile (input BatchNorm)
  auto fetch = [&](int tile) {
    const int img = tile / per_img;
    const int trem = tile - img * per_img;
    const int th = trem / p.tiles_w;
    const int oh0 = th * BH, ow0 = (trem - th * p.tiles_w) * 32;
    const int ibase = img * p.h;
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int i = threadIdx.x + u * NT;
      const int q = i / NPX, px = i - q * NPX;
      const int oh = oh0 + px / 32, ow = ow0 + (px & 31);
      const int co = co0 + 4 * q;
      const bool ok = i < NDY && oh < p.h && ow < p.w && co < p.cout;
      pdy[u] = load4(dr, ok ? (uint32_t)(((ibase + oh) * p.w + ow) * p.dy_ps + co) * 4u : kOOB);
    }
#pragma unroll
    for (int u = 0; u < NX; ++u) {
      const int i = threadIdx.x + u * NT;
      const int q = i / LPX, hp = i - q * LPX;
      const int lr = hp / LW, lc = hp - lr * LW;
      const int ih = oh0 - HALO + lr, iw = ow0 - HALO + lc;
      const int c = c0 + 4 * q;
      const bool ok = i < xtotal && (unsigned)ih < (unsigned)p.h && (unsigned)iw < (unsigned)p.w;
      pxx[u] = load4(xr, ok ? (uint32_t)(((ibase + ih) * p.w + iw) * p.x_ps + c) * 4u : kOOB);
      xok = u == 0 ? (uint32_t)ok : (xok | ((uint32_t)ok << u));
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int i = threadIdx.x + u * NT;
      if (NDY % NT != 0 && i >= NDY) break;
      const int q = i / NPX, px = i - q * NPX;
      const int co = co0 + 4 * q;
#pragma unroll
      for (int k = 0; k < 4; ++k) dyt[(4 * q + k) * DYS + px] = co + k < p.cout ? pdy[u][k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < NX; ++u) {
      const int i = threadIdx.x + u * NT;
      if (i < xtotal) {
        const int q = i / LPX, hp = i - q * LPX;
        const int c = c0 + 4 * q;
        if (p.isave && ((xok >> u) & 1u)) ibn_apply(pxx[u], q);
#pragma unroll
        for (int k = 0; k < 4; ++k) xt[(4 * q + k) * LPX + hp] = c + k < p.cin ? pxx[u][k] : 0.f;
      }
    }
  };
  if (PF && tb < te) fetch(tb);
  for (int tile = tb; tile < te; ++tile) {
    __syncthreads();  // the previous tile's fragment reads are done
    if (PF) {
      store();
    } else {  // lower register footprint: dY at once, X in batches of 4 loads per thread
      const int img = tile / per_img;
      const int trem = tile - img * per_img;
      const int th = trem / p.tiles_w;
      const int oh0 = th * BH, ow0 = (trem - th * p.tiles_w) * 32;
      const int ibase = img * p.h;
      {
        f4 v[NI];
#pragma unroll
        for (int u = 0; u < NI; ++u) {
          const int i = threadIdx.x + u * NT;
          const int q = i / NPX, px = i - q * NPX;
          const int oh = oh0 + px / 32, ow = ow0 + (px & 31);
          const int co = co0 + 4 * q;
          const bool ok = i < NDY && oh < p.h && ow < p.w && co < p.cout;
          v[u] = load4(dr, ok ? (uint32_t)(((ibase + oh) * p.w + ow) * p.dy_ps + co) * 4u : kOOB);
        }
#pragma unroll
        for (int u = 0; u < NI; ++u) {
          const int i = threadIdx.x + u * NT;
          if (NDY % NT != 0 && i >= NDY) break;
          const int q = i / NPX, px = i - q * NPX;
          const int co = co0 + 4 * q;
#pragma unroll
          for (int k = 0; k < 4; ++k)
            dyt[(4 * q + k) * DYS + px] = co + k < p.cout ? v[u][k] : 0.f;
        }
      }
      for (int i0 = threadIdx.x; i0 < xtotal; i0 += 4 * NT) {
        f4 v[4];
        bool okv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = i0 + u * NT;
          const int q = i / LPX, hp = i - q * LPX;
          const int lr = hp / LW, lc = hp - lr * LW;
          const int ih = oh0 - HALO + lr, iw = ow0 - HALO + lc;
          const int c = c0 + 4 * q;
          const bool ok =
              i < xtotal && (unsigned)ih < (unsigned)p.h && (unsigned)iw < (unsigned)p.w;
          okv[u] = ok;
          v[u] = load4(xr, ok ? (uint32_t)(((ibase + ih) * p.w + iw) * p.x_ps + c) * 4u : kOOB);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = i0 + u * NT;
          if (i >= xtotal) break;
          const int q = i / LPX, hp = i - q * LPX;
          const int c = c0 + 4 * q;
          if (p.isave && okv[u]) ibn_apply(v[u], q);
#pragma unroll
          for (int k = 0; k < 4; ++k) xt[(4 * q + k) * LPX + hp] = c + k < p.cin ? v[u][k] : 0.f;
        }
      }
    }
    __syncthreads();
    if (PF && tile + 1 < te) fetch(tile + 1);
    auto frag = [&](int ch, f4* fa, f4* fb) {
      const int px0 = ch * 16 + 4 * g;
      const int poff = (px0 >> 5) * LW + (px0 & 31);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const f4*>(&dyt[(i * 16 + r) * DYS + px0]);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* b = &xt[bbase[j] + poff];
        if (KS == 1) fb[j] = *reinterpret_cast<const f4*>(b);  // 16-byte aligned: no tap shift
        else fb[j] = f4{b[0], b[1], b[2], b[3]};
      }
    };
    if (!BF) {
#pragma unroll 2
      for (int ch = 0; ch < NPX / 16; ++ch) {
        f4 fa[TM], fb[TN];
        frag(ch, fa, fb);
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s2], fb[j][s2], acc[i][j], 0, 0, 0);
        if constexpr (NR > 0) {  // this lane's 4 pixels x its columns, remainder rows
          const int px0 = ch * 16 + 4 * g;
#pragma unroll
          for (int q = 0; q < NR; ++q) {
            const f4 d = *reinterpret_cast<const f4*>(&dyt[(16 * TM + q) * DYS + px0]);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              racc[j][q] = __builtin_fmaf(d[0], fb[j][0], racc[j][q]);
              racc[j][q] = __builtin_fmaf(d[1], fb[j][1], racc[j][q]);
              racc[j][q] = __builtin_fmaf(d[2], fb[j][2], racc[j][q]);
              racc[j][q] = __builtin_fmaf(d[3], fb[j][3], racc[j][q]);
            }
          }
        }
      }
    } else {  // bf16 operands: one 16x16x32 MFMA per pair of 16-pixel chunks
#pragma unroll 2
      for (int ch = 0; ch < NPX / 16; ch += 2) {
        f4 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
        frag(ch, fa0, fb0);
        frag(ch + 1, fa1, fb1);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                pack_bf16(fa0[i], fa1[i]), pack_bf16(fb0[j], fb1[j]), acc[i][j], 0, 0, 0);
      }
    }
  }

  const int ncol4 = TAPS * p.cin4;
  float* out = p.part + (int64_t)blockIdx.x * p.cout * ncol4;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = (wave * TN + j) * 16 + r;
    const int t = n / p.csw;
    const int cl = n - t * p.csw;
    if (t >= TAPS || cl >= csw_real) continue;
    const int col = t * p.cin4 + c0 + cl;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + i * 16 + g * 4 + e;
        if (co < p.cout) out[(int64_t)co * ncol4 + col] = acc[i][j][e];
      }
  }
  if constexpr (NR > 0) {  // the 4 lane groups' pixel sums (fixed order), rows 16*TM + q
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = (wave * TN + j) * 16 + r;
      const int t = n / p.csw;
      const int cl = n - t * p.csw;
#pragma unroll
      for (int q = 0; q < NR; ++q) {
        float v = racc[j][q];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (g == 0 && t < TAPS && cl < csw_real)
          out[(int64_t)(co0 + 16 * TM + q) * ncol4 + t * p.cin4 + c0 + cl] = v;
      }
    }
  }
}

#if VAE2_PART(3)
// dw[co][ci][kh][kw] (+)= sum_s part[s][co][(kh*k+kw)*cin4 + ci]
// Block = 32 slab columns x 8 split groups: thread (g, col) sums splits g, g+8, ...
// (unrolled: its loads are independent), the 8 group sums are combined in LDS in a fixed
// order (deterministic).  Small slabs still get ceil(slab/32) blocks and short chains.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part,
                                                           int splits, int cout, int cin,
                                                           int cin4, int k,
                                                           float* __restrict__ dw, int64_t ld,
                                                           int accumulate) {
  __shared__ float red[8][32];
  const int kk = k * k;
  const int ncol4 = kk * cin4;
  const int total = cout * ncol4;  // slab elements
  const int cl = threadIdx.x & 31, sg = threadIdx.x >> 5;
  const int idx = blockIdx.x * 32 + cl;
  float s = 0.f;
  if (idx < total) {
    const float* src = part + idx;
    const int64_t stride = (int64_t)total;
#pragma unroll 8
    for (int sp = sg; sp < splits; sp += 8) s += src[sp * stride];
  }
  red[sg][cl] = s;
  __syncthreads();
  if (sg != 0 || idx >= total) return;
  s = red[0][cl];
#pragma unroll
  for (int j = 1; j < 8; ++j) s += red[j][cl];
  const int co = idx / ncol4;
  const int col = idx - co * ncol4;
  const int t = col / cin4;
  const int ci = col - t * cin4;
  if (ci >= cin) return;
  const int64_t o = (int64_t)co * ld + ci * kk + t;
  dw[o] = accumulate ? dw[o] + s : s;
}

#endif  // VAE2_PART(3)
// Deferred reductions (vae2_wgrad_defer / vae2_wgrad_flush): the weight gradients of
// one BatchNorm depth level (the lock-stepped branch convs, a head's branch blocks) share
// one reduce launch; blocks are partitioned between the jobs by prefix.
struct WRJob {
  const float* part;
  float* dw;
  int64_t ld;
  int splits, cout, cin, cin4, k, accumulate, blk0;
};
constexpr int kWrMaxJobs = 32;  // (kernel argument: 32 x 56 B)
struct WRMulti {
  WRJob j[kWrMaxJobs];
  int n;
};

#if VAE2_PART(3)
__global__ __launch_bounds__(256) void wgrad_reduce_multi_kernel(WRMulti m) {
  int i = 0;
  while (i + 1 < m.n && (int)blockIdx.x >= m.j[i + 1].blk0) ++i;
  const WRJob& J = m.j[i];
  __shared__ float red[8][32];
  const int kk = J.k * J.k;
  const int ncol4 = kk * J.cin4;
  const int total = J.cout * ncol4;
  const int cl = threadIdx.x & 31, sg = threadIdx.x >> 5;
  const int idx = ((int)blockIdx.x - J.blk0) * 32 + cl;
  float s = 0.f;
  if (idx < total) {
    const float* src = J.part + idx;
    const int64_t stride = (int64_t)total;
#pragma unroll 8
    for (int sp = sg; sp < J.splits; sp += 8) s += src[sp * stride];
  }
  red[sg][cl] = s;
  __syncthreads();
  if (sg != 0 || idx >= total) return;
  s = red[0][cl];
#pragma unroll
  for (int q = 1; q < 8; ++q) s += red[q][cl];
  const int co = idx / ncol4;
  const int col = idx - co * ncol4;
  const int t = col / J.cin4;
  const int ci = col - t * J.cin4;
  if (ci >= J.cin) return;
  const int64_t o = (int64_t)co * J.ld + ci * kk + t;
  J.dw[o] = J.accumulate ? J.dw[o] + s : s;
}

#endif  // VAE2_PART(3)

struct WRQueued {
  WRJob job;
  hipStream_t stream;
};
// the deferral switch is per thread (set inside the calling thread's backward functions);
// the queue is shared, so the end-of-backward flush may run on any thread
static thread_local bool g_wr_defer = false;
static std::vector<WRQueued> g_wr_queue;
static std::mutex g_wr_mu;

struct WTile {
  int tm, tn, gx, gy, splits, px_split;
};

static WTile pick_wtile(int64_t P, int cout, int ncol4) {
  WTile t;
  int mt = (cout + 15) / 16;
  t.tm = mt <= 4 ? mt : 4;
  t.gy = (int)ceil_div(cout, 16 * t.tm);
  int ct = (ncol4 + 15) / 16;
  // tune key 1: when 4 row tiles would leave a third-empty second column block (ct = 4:
  // 64 columns as 48 + 48), take 2 row tiles and all 64 columns in one block instead
  if (g_wgrad_cols && t.tm == 4 && ct == 4) {
    t.tm = 2;
    t.gy = (int)ceil_div(cout, 32);
  }
  const int tn_max = t.tm == 4 ? 3 : 4;  // <4,4> would not fit 2 waves/SIMD without spills
  t.tn = ct <= tn_max ? ct : tn_max;
  t.gx = (int)ceil_div(ncol4, 16 * t.tn);
  int64_t tiles = (int64_t)t.gx * t.gy;
  // ~1024 workgroups (4 waves each; set_tune key 18), at least 256 pixels (4 chunks per
  // wave) each: small layers get enough workgroups in flight to hide the load latency
  // (512 / 256 measured 0.5 / 1.2 % slower in the step)
  int64_t want = ceil_div(g_wgrad_wgs, tiles);
  int64_t maxs = ceil_div(P, 256);
  int64_t s = want < maxs ? want : maxs;
  if (s < 1) s = 1;
  t.px_split = (int)(ceil_div(ceil_div(P, s), 64) * 64);
  t.splits = (int)ceil_div(P, t.px_split);
  return t;
}

#if VAE2_PART(3)
template <int TM, bool V4>
static void launch_wgrad_tn_v(const WGrad& p, int tn, dim3 grid, hipStream_t s) {
  const size_t lds = (size_t)3 * TM * 4 * 4 * 64 * sizeof(float) / 4 * tn;  // 3 waves x NV x 64
  switch (tn) {
#define CASE(T) \
  case T: \
    if (g_bf16) VAE2_LAUNCH((wgrad_kernel<TM, T, true, V4>), grid, dim3(256), lds, s, p); \
    else VAE2_LAUNCH((wgrad_kernel<TM, T, false, V4>), grid, dim3(256), lds, s, p); \
    break;
    CASE(1) CASE(2) CASE(3)
    default: CASE(4)
#undef CASE
  }
}

template <int TM>
static void launch_wgrad_tn(const WGrad& p, int tn, dim3 grid, hipStream_t s, bool v4) {
  if (v4) launch_wgrad_tn_v<TM, true>(p, tn, grid, s);
  else launch_wgrad_tn_v<TM, false>(p, tn, grid, s);
}

#endif  // VAE2_PART(3)

// ------------------------------------------------------------- checks ----
static bool conv_shapes_ok(const vae2_act* xd, const vae2_act* yd, int k, int stride, int pad) {
  if (!act_ok(xd) || !act_ok(yd)) return false;
  if (xd->n != yd->n) return false;
  if (k < 1 || stride < 1 || pad < 0) return false;
  int64_t oh = (xd->h + 2 * pad - k) / stride + 1;
  int64_t ow = (xd->w + 2 * pad - k) / stride + 1;
  return oh == yd->h && ow == yd->w;
}

static bool fits32(const vae2_act* d) {
  return d->n * d->h * d->w * d->ps < (int64_t(1) << 29);  // byte offsets < 2^31
}

// Bytes spanned by an activation view, for buffer descriptors.  With 16-byte
// aligned pixels (ps % 4 == 0) the last pixel's final 4-channel quad is included
// (it lies inside the pixel stride), so a whole-access range check never drops
// real channels of the last quad.
static uint32_t act_bytes(const vae2_act* d) {
  int64_t tail = (d->ps % 4 == 0) ? ((d->c + 3) / 4 * 4) : d->c;
  int64_t last = ((d->n * d->h * d->w) - 1) * d->ps + tail;
  return (uint32_t)(last * 4);
}

#if VAE2_PART(1)
// hipOccupancyMaxActiveBlocksPerMultiprocessor of gemm1x1_kernel<tm, tn> with `lds` bytes
// of dynamic LDS (cached per (tm, tn, lds)); at least 1.
int gemm1_blocks_per_cu(int tm, int tn, size_t lds) {
  static int cache[3][9][4] = {};
  static size_t cache_lds[3][9][4] = {};
  if (tn < 3 || tn > 8 || tm < 1 || tm > 2) return 1;
  for (int i = 0; i < 4; ++i)
    if (cache[tm][tn][i] && cache_lds[tm][tn][i] == lds) return cache[tm][tn][i];
  int n = 0;
  hipError_t e = hipErrorInvalidValue;
#define CASE(M, T)                                                                       \
  case T:                                                                                \
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(                                    \
        &n, reinterpret_cast<const void*>(gemm1x1_kernel<M, T>), 256, lds);              \
    break;
  if (tm == 1) {
    switch (tn) { CASE(1, 3) CASE(1, 4) CASE(1, 5) CASE(1, 6) CASE(1, 7) CASE(1, 8) }
  } else {
    switch (tn) { CASE(2, 3) CASE(2, 4) CASE(2, 5) CASE(2, 6) CASE(2, 7) CASE(2, 8) }
  }
#undef CASE
  if (e != hipSuccess || n < 1) {
    (void)hipGetLastError();
    n = 1;
  }
  for (int i = 0; i < 4; ++i)
    if (!cache[tm][tn][i]) {
      cache[tm][tn][i] = n;
      cache_lds[tm][tn][i] = lds;
      break;
    }
  return n;
}

int launch_gemm1(const float* a, const vae2_act* ad, const float* wp, uint32_t w_bytes,
                 const float* bias, float* y, const vae2_act* yd, float beta, float* stats,
                 const G1Tile& t, hipStream_t s, const char* fn, const float* bx, int bx_ps,
                 int brelu, const float* bsave, uint32_t bx_bytes) {
  // (16-byte stores of whole channel quads where y is aligned, 4-byte stores otherwise, so
  // the statistics rows vae2_conv2d_fwd_stats_rows reports do not depend on y's alignment;
  // statistics are of the fresh output only)
  if (stats && beta != 0.f) return -1;
  Gemm1 p{};
  p.bx = bx; p.bx_ps = bx_ps; p.brelu = brelu; p.bsave = bsave; p.bx_bytes = bx_bytes;
  p.vec = vec_ok(y, (int)yd->ps) ? 1 : 0;
  p.a = a; p.a_ps = (int)ad->ps; p.a_c = (int)ad->c; p.a_c4 = round_up((int)ad->c, 4);
  p.M = (int)act_pixels(yd);
  p.w = wp; p.n = (int)yd->c; p.bias = bias; p.y = y; p.y_ps = (int)yd->ps; p.beta = beta;
  p.stats = stats; p.a_bytes = act_bytes(ad); p.w_bytes = w_bytes;
  const dim3 grid((unsigned)t.grid_x, (unsigned)t.nblk);
#define CASE(M, T) \
  case T: VAE2_LAUNCH((gemm1x1_kernel<M, T>), grid, dim3(256), t.lds, s, p); break;
  if (t.tm == 1) {
    switch (t.tn) {
      CASE(1, 3) CASE(1, 4) CASE(1, 5) CASE(1, 6) CASE(1, 7) CASE(1, 8)
      default: return fail(fn, "gemm1x1: unsupported N block");
    }
  } else {
    switch (t.tn) {
      CASE(2, 3) CASE(2, 4) CASE(2, 5) CASE(2, 6) CASE(2, 7) CASE(2, 8)
      default: return fail(fn, "gemm1x1: unsupported N block");
    }
  }
#undef CASE
  return check_launch(fn);
}

#endif  // VAE2_PART(1)

}  // namespace vae2

using namespace vae2;

// ---------------------------------------------- direct 3x3: host dispatch ----

struct DTile {
  int tm, tn, nblk, cs4, tiles_h, tiles_w;
  int nr = 0;  // output channels on the VALU beside the MFMA tiles (dconv3_body NR)
  int nw = 4;  // waves per workgroup (dconv3_body NW); tile rows = nw * tm / 2
  int ks = 1;  // K shares over 4-wave sets (dconv3_body KS, nw = 4 ks, tile rows = 2 tm)
};


static bool dconv_legal(const vae2_act* ad, const vae2_act* yd, int k, int stride, int pad,
                        const float* a) {
  return k == 3 && stride == 1 && pad == 1 && ad->h == yd->h && ad->w == yd->w &&
         vec_ok(a, (int)ad->ps);
}

// remainder = true: an N of 16*TN + NR with (TN, NR) = (1, 2), (2, 4) or (4, 8) (the 18 /
// 36 / 72-channel branches) takes TN MFMA tiles plus NR VALU channels in one N block
// (fp32 operands only).
static DTile pick_dtile(const vae2_act* ad, const vae2_act* yd, bool remainder = true) {
  DTile d;
  Tile t = pick_tile(act_pixels(yd), (int)yd->c);
  d.tn = t.tn;
  d.nblk = t.nblk;
  const int N = (int)yd->c, tn = N / 16, nr = N % 16;
  // (auto: all three where the single N block still fills the chip twice -- in the
  //  concurrent training step the 32 + 4 form is 0.4 % faster than the padded 48-column
  //  tiles; set_algo bit 128 restricts auto to 16 + 2; algo 2 takes all three wherever
  //  legal, for the tests)
  if (remainder && g_dconv_nr && !g_bf16 &&
      ((tn == 1 && nr == 2) ||
       ((g_conv_algo == 2 || g_dconv_nr_wide) && ((tn == 2 && nr == 4) || (tn == 4 && nr == 8))))) {
    d.tn = tn;
    d.nr = nr;
    d.nblk = 1;
  }
  const int Q = round_up((int)ad->c, 4) / 4;
  const int nsl = (Q + kDcMaxCs4 - 1) / kDcMaxCs4;
  d.cs4 = (Q + nsl - 1) / nsl;  // balanced slabs
  d.tiles_w = (int)ceil_div(yd->w, kDcBW);
  // 8-row tiles unless that leaves fewer than ~3 workgroups per CU
  d.tm = 4;
  // (from the all-MFMA N blocking, so the tile rows and the BN partial-statistics rows
  //  do not depend on the remainder switch or the grouped path)
  if (yd->h < 8 || ad->n * ceil_div(yd->h, 8) * d.tiles_w * t.nblk < 768) d.tm = 2;
  // tune key 2: the 8-row tiles as 8 waves of one row each (TM = 2, NW = 8) -- same tile
  // rows, so the same BN partial-statistics rows
  if (g_dconv_nw8 && d.tm == 4 && !g_bf16) {
    d.tm = 2;
    d.nw = 8;
  }
  d.tiles_h = (int)ceil_div(yd->h, d.nw * d.tm / 2);
  // the remainder form has one N block: only where the tiles alone fill the chip twice
  // (algo 2 forces it wherever legal, for the tests)
  if (d.nr && g_conv_algo != 2 && ad->n * d.tiles_h * d.tiles_w < 512) {
    d.tn = t.tn; d.nblk = t.nblk; d.nr = 0;
  }
  // tune key 13: a layer whose tiles leave fewer than 2 workgroups per CU (the 72-channel
  // branch at 32 x 64: 256 workgroups = one wave per SIMD) takes 16-channel N blocks --
  // more workgroups re-staging the same halo tile (L2-resident) for more waves per SIMD
  if (g_dconv_n16 && !g_bf16 && d.nr == 0 && d.tn > 1 && N > 16 &&
      ad->n * d.tiles_h * d.tiles_w * d.nblk < 512) {
    d.tn = 1;
    d.nblk = (N + 15) / 16;
  }
  // tune key 14: the 72-channel branch as two N blocks of 32 MFMA + 4 VALU channels
  // (block b: channels 36 b ..) -- the same workgroups as the two padded 48-column blocks
  // (24 of their 96 MFMA columns are padding), a third fewer MFMAs per block
  if (remainder && g_dconv_split72 && g_dconv_nr && !g_bf16 && d.nr == 0 && N == 72 &&
      d.nblk == 2 && d.tn == 3) {
    d.tn = 2;
    d.nr = 4;
  }
  // tune key 15: 4-row tiles (TM = 2) that leave at most 2 workgroups per CU run as 8-wave
  // workgroups splitting K in two -- the same tiles, rows and statistics rows, twice the
  // waves per SIMD (the 72-channel branch at 32 x 64: 256 workgroups, one wave per SIMD;
  // conv_bench 25.4 / 24.9 -> 25.0 / 24.6 us fwd / dgrad, step 902.1 / 900.7 -> 908.6 / 910.3
  // frames/s over 2 A/B pairs, scripts/gpu_r6_n.sh)
  if (g_dconv_ksp && !g_bf16 && d.nr == 0 && d.tm == 2 && d.nw == 4 && d.tn >= 2 &&
      ad->n * d.tiles_h * d.tiles_w * d.nblk < 512) {
    d.ks = g_dconv_ksp == 2 ? 4 : 2;
    d.nw = 4 * d.ks;
  }
  return d;
}

// The streaming kernel (dconv_stream.hip) takes the 18 -> 18 and 36 -> 36 direct convs
// (fp32 operands, the VALU-remainder form) wherever the direct kernel is legal: its
// partial-statistics rows are its workgroups, so dconv_rows asks the same predicate.
static bool stream_use(const vae2_act* ad, const vae2_act* yd) {
  return g_dconv_stream && !g_bf16 && g_dconv_nr && g_conv_algo != 1 &&
         (g_conv_algo == 2 || ad->w >= 16) && dconv3s_shape(ad, yd);
}

static bool dconv_use(const vae2_act* ad, const vae2_act* yd, int k, int stride, int pad,
                      const float* a) {
  if (g_conv_algo == 1 || !dconv_legal(ad, yd, k, stride, pad, a)) return false;
  if (g_conv_algo == 2 || stream_use(ad, yd)) return true;
  // auto: enough workgroups to fill the chip (narrow images waste partial 32-column
  // tiles and low-resolution layers have too few tiles: the gather kernel wins there)
  DTile d = pick_dtile(ad, yd, false);
  return ad->w >= 16 && ad->n * d.tiles_h * d.tiles_w * d.nblk >= 256;
}

// BatchNorm fused at a direct-3x3 conv's input (DConv::isave / irelu) or, for its data
// gradient, that BatchNorm's backward partials in the epilogue (DConv::bx ...).
struct BnSide {
  const float* isave = nullptr;
  int irelu = 0;
  const float* bx = nullptr;
  int bx_ps = 0, brelu = 0;
  const float* bsave = nullptr;
  uint32_t bx_bytes = 0;
};

int launch_dconv(const float* a, const vae2_act* ad, const float* wp, uint32_t w_bytes,
                 const float* bias, float* y, const vae2_act* yd, float beta,
                 float* stats, bool flip, hipStream_t s, const char* fn,
                 const BnSide& bn = BnSide{});

#if VAE2_PART(2)
template <int TM, bool FLIP, int NW = 4>
static void dconv_launch_tn(const DConv& p, int tn, dim3 grid, size_t shm, hipStream_t s,
                            int nr = 0) {
  if (p.isave || p.bx) {  // fused BatchNorm (fp32 operands): forward input / dgrad partials
    constexpr int X = FLIP ? 2 : 1;
    if (nr) {
      if (tn == 1 && nr == 2) VAE2_LAUNCH((dconv3_kernel<TM, 1, FLIP, false, 2, X, NW>), grid, dim3(64 * NW), shm, s, p);
      else if (tn == 2 && nr == 4) VAE2_LAUNCH((dconv3_kernel<TM, 2, FLIP, false, 4, X, NW>), grid, dim3(64 * NW), shm, s, p);
      else VAE2_LAUNCH((dconv3_kernel<TM, 4, FLIP, false, 8, X, NW>), grid, dim3(64 * NW), shm, s, p);
      return;
    }
    switch (tn) {
#define CASE(T) \
  case T: VAE2_LAUNCH((dconv3_kernel<TM, T, FLIP, false, 0, X, NW>), grid, dim3(64 * NW), shm, s, p); break;
      CASE(1) CASE(2) CASE(3) CASE(4)
#undef CASE
    }
    return;
  }
  if (nr) {  // fp32 operands (pick_dtile)
    if (tn == 1 && nr == 2) VAE2_LAUNCH((dconv3_kernel<TM, 1, FLIP, false, 2, 0, NW>), grid, dim3(64 * NW), shm, s, p);
    else if (tn == 2 && nr == 4) VAE2_LAUNCH((dconv3_kernel<TM, 2, FLIP, false, 4, 0, NW>), grid, dim3(64 * NW), shm, s, p);
    else VAE2_LAUNCH((dconv3_kernel<TM, 4, FLIP, false, 8, 0, NW>), grid, dim3(64 * NW), shm, s, p);
    return;
  }
  switch (tn) {
#define CASE(T) \
  case T:                                                                         \
    if (g_bf16) VAE2_LAUNCH((dconv3_kernel<TM, T, FLIP, true, 0, 0, NW>), grid, dim3(64 * NW), shm, s, p); \
    else VAE2_LAUNCH((dconv3_kernel<TM, T, FLIP, false, 0, 0, NW>), grid, dim3(64 * NW), shm, s, p);        \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4)
#undef CASE
  }
}

// K-split form (pick_dtile, set_tune key 15): TM = 2, 4 KS waves, fp32 operands, no remainder
template <bool FLIP, int KS>
static void dconv_launch_ksp(const DConv& p, int tn, dim3 grid, size_t shm, hipStream_t s) {
  constexpr int X = FLIP ? 2 : 1, NW = 4 * KS;
  const bool bn = p.isave || p.bx;
  switch (tn) {
#define CASE(T)                                                                                        \
  case T:                                                                                              \
    if (bn) VAE2_LAUNCH((dconv3_kernel<2, T, FLIP, false, 0, X, NW, KS>), grid, dim3(64 * NW), shm, s, p); \
    else VAE2_LAUNCH((dconv3_kernel<2, T, FLIP, false, 0, 0, NW, KS>), grid, dim3(64 * NW), shm, s, p);    \
    break;
    CASE(2) CASE(3) CASE(4)
#undef CASE
  }
}

#endif  // VAE2_PART(2)

static DConv make_dconv(const DTile& d, const float* a, const vae2_act* ad, const float* wp,
                        uint32_t w_bytes, const float* bias, float* y, const vae2_act* yd,
                        float beta, float* stats) {
  DConv p{};
  p.a = a; p.a_ps = (int)ad->ps; p.a_c = (int)ad->c; p.a_c4 = round_up((int)ad->c, 4);
  p.img_h = (int)ad->h; p.img_w = (int)ad->w;
  p.tiles_h = d.tiles_h; p.tiles_w = d.tiles_w; p.cs4 = d.cs4;
  p.w = wp; p.a_bytes = act_bytes(ad); p.w_bytes = w_bytes;
  p.n = (int)yd->c; p.bias = bias; p.y = y; p.y_ps = (int)yd->ps; p.beta = beta;
  p.stats = stats;
  p.vec_out = g_vec_out && vec_ok(y, (int)yd->ps) && !(stats && beta != 0.f);
  return p;
}

static size_t dconv_shm(const DTile& d) {
  const int rows = (d.ks > 1 ? 4 : d.nw) * d.tm / 2;  // output rows of a tile (KS: 4 row waves)
  const size_t stage = ((size_t)(rows + 2) * (kDcBW + 2) * (d.cs4 * 4 + 4) +
                        (size_t)d.nr * ((9 * d.cs4 + 7) / 8) * 32 + 2 * kDcTab) * sizeof(float);
  // KS > 1: shares 1 .. KS-1's accumulators ([KS - 1][4 waves][TM][TN][64] f4) in the same
  // LDS after the K loop
  const size_t kred = (size_t)(d.ks - 1) * 4 * d.tm * d.tn * 64 * 16;
  return stage > kred ? stage : kred;
}

#if VAE2_PART(2)
template <int TM, bool FLIP>
static void dconv_group_launch_tn(const DConvGroup& g, int tn, dim3 grid, size_t shm,
                                  hipStream_t s) {
  switch (tn) {
#define CASE(T)                                                                          \
  case T:                                                                                \
    if (g_bf16) VAE2_LAUNCH((dconv3_group_kernel<TM, T, FLIP, true>), grid, dim3(256), shm, s, g); \
    else VAE2_LAUNCH((dconv3_group_kernel<TM, T, FLIP>), grid, dim3(256), shm, s, g);    \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4)
#undef CASE
  }
}

int launch_dconv(const float* a, const vae2_act* ad, const float* wp, uint32_t w_bytes,
                 const float* bias, float* y, const vae2_act* yd, float beta,
                 float* stats, bool flip, hipStream_t s, const char* fn, const BnSide& bn) {
  if (stream_use(ad, yd)) {
    dconv3s_launch(a, ad, wp, w_bytes, bias, y, yd, beta, stats, flip, bn.isave, bn.irelu,
                   bn.bx, bn.bx_ps, bn.brelu, bn.bsave, bn.bx_bytes, act_bytes(ad), s);
    return check_launch(fn);
  }
  DTile d = pick_dtile(ad, yd);
  DConv p{};
  p.a = a; p.a_ps = (int)ad->ps; p.a_c = (int)ad->c; p.a_c4 = round_up((int)ad->c, 4);
  p.img_h = (int)ad->h; p.img_w = (int)ad->w;
  p.tiles_h = d.tiles_h; p.tiles_w = d.tiles_w; p.cs4 = d.cs4;
  p.w = wp; p.a_bytes = act_bytes(ad); p.w_bytes = w_bytes;
  p.n = (int)yd->c; p.bias = bias; p.y = y; p.y_ps = (int)yd->ps; p.beta = beta;
  p.stats = stats;
  p.isave = bn.isave; p.irelu = bn.irelu;
  p.bx = bn.bx; p.bx_ps = bn.bx_ps; p.brelu = bn.brelu; p.bsave = bn.bsave;
  p.bx_bytes = bn.bx_bytes;
  p.vec_out = g_vec_out && vec_ok(y, (int)yd->ps) && !(stats && beta != 0.f);
  dim3 grid((unsigned)(ad->n * d.tiles_h * d.tiles_w), (unsigned)d.nblk);
  const size_t shm = dconv_shm(d);
  if (d.ks == 4) {
    if (flip) dconv_launch_ksp<true, 4>(p, d.tn, grid, shm, s);
    else dconv_launch_ksp<false, 4>(p, d.tn, grid, shm, s);
  } else if (d.ks == 2) {
    if (flip) dconv_launch_ksp<true, 2>(p, d.tn, grid, shm, s);
    else dconv_launch_ksp<false, 2>(p, d.tn, grid, shm, s);
  } else if (d.nw == 8) {
    if (flip) dconv_launch_tn<2, true, 8>(p, d.tn, grid, shm, s, d.nr);
    else dconv_launch_tn<2, false, 8>(p, d.tn, grid, shm, s, d.nr);
  } else if (d.tm == 4) {
    if (flip) dconv_launch_tn<4, true>(p, d.tn, grid, shm, s, d.nr);
    else dconv_launch_tn<4, false>(p, d.tn, grid, shm, s, d.nr);
  } else {
    if (flip) dconv_launch_tn<2, true>(p, d.tn, grid, shm, s, d.nr);
    else dconv_launch_tn<2, false>(p, d.tn, grid, shm, s, d.nr);
  }
  return check_launch(fn);
}

#endif  // VAE2_PART(2)

static int64_t dconv_rows(const vae2_act* ad, const vae2_act* yd) {
  if (stream_use(ad, yd)) return dconv3s_rows(ad, yd);
  DTile d = pick_dtile(ad, yd);
  return ad->n * d.tiles_h * d.tiles_w;
}

// ---------------------------------------- direct 3x3 wgrad: host dispatch ----
struct W3Tile {
  int ks, tm, tn, bh, csw, n_ci_slabs, n_co_slabs, tiles_h, tiles_w, ntiles, tps, splits;
  bool pf;
  int nr = 0;  // output channels on the VALU beside the MFMA rows (wgrad3_kernel NR)
  int nw = 4;  // waves per workgroup (wgrad3_kernel NW)
};

// Resident workgroups per CU of the wgrad3_kernel instance a tile selects (PART(3): the
// launch dispatch run in probe mode + hipOccupancyMaxActiveBlocksPerMultiprocessor).
int wgrad3_blocks_per_cu(const W3Tile& t, size_t lds);
static size_t wgrad3_lds(const W3Tile& t);

static bool wgrad3_shape_ok(const vae2_act* xd, const vae2_act* dyd, int k, int stride, int pad) {
  // (the KS = 1 form of the kernel measured slower than the gather kernel on 1x1 convs:
  //  without the 9-tap reuse the staging does not pay for itself)
  return k == 3 && pad == 1 && stride == 1 && xd->h == dyd->h &&
         xd->w == dyd->w && xd->ps % 4 == 0 && dyd->ps % 4 == 0 && dyd->w >= 16;
}

static W3Tile pick_w3tile(const vae2_act* xd, const vae2_act* dyd, int k) {
  W3Tile t;
  t.ks = k;
  const int cin4 = round_up((int)xd->c, 4);
  const int maxc = k == 1 ? 64 : 36;  // channels per slab (columns = taps x channels)
  int nsl = (cin4 + maxc - 1) / maxc;
  t.csw = round_up((int)ceil_div(cin4, nsl), 4);
  t.n_ci_slabs = (int)ceil_div(cin4, t.csw);
  const int nt = (k * k * t.csw + 15) / 16;
  t.tn = (nt + 3) / 4;
  const int mt = (int)((dyd->c + 15) / 16);
  t.n_co_slabs = (mt + 3) / 4;
  t.tm = (mt + t.n_co_slabs - 1) / t.n_co_slabs;
  // 18 / 36 / 72 output channels: co slabs of 16 + 2, 32 + 4, 2 x (32 + 4): MFMA rows
  // plus VALU rows (fp32 operands)
  if (k == 3 && g_dconv_nr && !g_bf16 && (dyd->c == 18 || dyd->c == 36 || dyd->c == 72)) {
    t.tm = dyd->c == 18 ? 1 : 2;
    t.nr = dyd->c == 18 ? 2 : 4;
    t.n_co_slabs = (int)(dyd->c / (16 * t.tm + t.nr));
  }
  // tune key 3: the remainder layers' column tiles over 8 waves (twice the waves per SIMD)
  if (g_wgrad_nw8 && t.nr && !g_bf16) {
    const int tn2 = (nt + 7) / 8;
    if ((t.tm == 1 && tn2 == 2) || (t.tm == 2 && tn2 == 3)) {
      t.tn = tn2;
      t.nw = 8;
    }
  }
  t.bh = (t.tm <= 2 && t.csw <= 24 && k == 3) ? 8 : 4;
  t.tiles_h = (int)ceil_div(dyd->h, t.bh);
  t.tiles_w = (int)ceil_div(dyd->w, 32);
  t.ntiles = (int)(dyd->n * t.tiles_h * t.tiles_w);
  const int gy = t.n_ci_slabs * t.n_co_slabs;
  // ~1024 workgroups in all and at most ~48 MB of partial slabs; layers with >= 1024
  // tile-slabs use >= 2 tiles per workgroup and prefetch tile t+1 while t computes
  int64_t want = ceil_div(1024, gy);
  const int64_t slab = (int64_t)dyd->c * k * k * cin4 * 4;
  const int64_t cap = 48ll << 20;
  if (want * slab > cap) want = cap / slab > 0 ? cap / slab : 1;
  if (want > t.ntiles) want = t.ntiles;
  t.tps = (int)ceil_div(t.ntiles, want);
  t.pf = (int64_t)t.ntiles * gy >= 1024;
  if (t.pf) {
    // one wave of workgroups: exactly as many as are resident at once (no straggler wave);
    // the residency comes from the instance's registers / LDS (the 18-channel 8-wave form
    // holds 145 VGPRs: one 512-thread workgroup per CU, not the 2 assumed before)
    const int64_t resident = 256 * (int64_t)wgrad3_blocks_per_cu(t, wgrad3_lds(t));
    int64_t w2 = resident / gy > 0 ? resident / gy : 1;
    if (w2 * slab > cap) w2 = cap / slab > 0 ? cap / slab : 1;
    t.tps = (int)ceil_div(t.ntiles, w2);
    if (t.tps < 2) t.tps = 2;
  }
  // at least 2 tiles per split: half the partial dW slabs (written here, read back by the
  // end-of-backward reductions) -- 36 -> 36 at 64x128 wrote 24 MB of slabs per launch,
  // 2.5x its dY.  In the concurrent training step: 814.7 -> 822.6 frames/s (A/B, same
  // box); 4 tiles per split: 789
  if (t.tps < 2) t.tps = 2;
  t.splits = (int)ceil_div(t.ntiles, t.tps);
  return t;
}

static size_t wgrad3_lds(const W3Tile& t) {
  const int npx = t.bh * 32, lpx = (t.bh + t.ks - 1) * (32 + t.ks - 1);
  const int rows = 16 * t.tm + 4 * ((t.nr + 3) / 4);
  return ((size_t)rows * (npx + 4) + (size_t)(t.csw + 1) * lpx) * sizeof(float);
}

#if VAE2_PART(3)
// Probe mode of the wgrad3 dispatch: record the instance (and its block size) instead of
// launching it.
struct W3Probe {
  bool on = false;
  const void* fn = nullptr;
  unsigned threads = 0;
};
static thread_local W3Probe g_w3probe;
#define W3_LAUNCH(K, GRID, BLOCK, SHM, S, ...)                         \
  do {                                                                \
    if (g_w3probe.on) {                                               \
      g_w3probe.fn = reinterpret_cast<const void*>(K);                \
      g_w3probe.threads = dim3(BLOCK).x;                              \
    } else {                                                          \
      VAE2_LAUNCH(K, GRID, BLOCK, SHM, S, __VA_ARGS__);               \
    }                                                                 \
  } while (0)

template <int TM, int BH, bool PF>
static void wgrad3_launch_tn(const WGrad3& p, int tn, int ks, dim3 grid, size_t shm,
                             hipStream_t s, int nr = 0, int nw = 4) {
  if constexpr (TM == 1 || TM == 2) {
    if (nr && nw == 8) {  // 8 waves: (TM, TN) = (1, 2) or (2, 3) (pick_w3tile)
      constexpr int R = TM == 1 ? 2 : 4, T8 = TM == 1 ? 2 : 3;
      W3_LAUNCH((wgrad3_kernel<TM, T8, BH, PF, 3, false, R, 8>), grid, dim3(512), shm, s, p);
      return;
    }
    if (nr) {  // (TM, NR) = (1, 2) or (2, 4): pick_w3tile, fp32 operands
      constexpr int R = TM == 1 ? 2 : 4;
      switch (tn) {
#define CASE(T) \
  case T: W3_LAUNCH((wgrad3_kernel<TM, T, BH, PF, 3, false, R>), grid, dim3(256), shm, s, p); break;
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6)
#undef CASE
      }
      return;
    }
  }
  if (ks == 1) {  // 1x1: at most 64 channels = 4 column tiles per slab, one per wave
    if (g_bf16) W3_LAUNCH((wgrad3_kernel<TM, 1, BH, PF, 1, true>), grid, dim3(256), shm, s, p);
    else W3_LAUNCH((wgrad3_kernel<TM, 1, BH, PF, 1>), grid, dim3(256), shm, s, p);
    return;
  }
  switch (tn) {
#define CASE(T) \
  case T:                                                                         \
    if (g_bf16) W3_LAUNCH((wgrad3_kernel<TM, T, BH, PF, 3, true>), grid, dim3(256), shm, s, p); \
    else W3_LAUNCH((wgrad3_kernel<TM, T, BH, PF, 3>), grid, dim3(256), shm, s, p);   \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6)
#undef CASE
  }
}

template <int BH, bool PF>
static void wgrad3_launch_tm(const WGrad3& p, const W3Tile& t, dim3 grid, size_t shm,
                             hipStream_t s) {
  switch (t.tm) {
    case 1: wgrad3_launch_tn<1, BH, PF>(p, t.tn, t.ks, grid, shm, s, t.nr, t.nw); break;
    case 2: wgrad3_launch_tn<2, BH, PF>(p, t.tn, t.ks, grid, shm, s, t.nr, t.nw); break;
    case 3: wgrad3_launch_tn<3, BH, PF>(p, t.tn, t.ks, grid, shm, s); break;
    default: wgrad3_launch_tn<4, BH, PF>(p, t.tn, t.ks, grid, shm, s); break;
  }
}

template <int BH>
static void wgrad3_launch(const WGrad3& p, const W3Tile& t, dim3 grid, size_t shm,
                          hipStream_t s) {
  if (t.pf) wgrad3_launch_tm<BH, true>(p, t, grid, shm, s);
  else wgrad3_launch_tm<BH, false>(p, t, grid, shm, s);
}

int wgrad3_blocks_per_cu(const W3Tile& t, size_t lds) {
  struct Key {
    int tm, tn, bh, ks, nr, nw, pf, bf;
    size_t lds;
    int n;
  };
  static Key cache[32];
  static int ncache = 0;
  const int bf = g_bf16;
  for (int i = 0; i < ncache; ++i) {
    const Key& k = cache[i];
    if (k.tm == t.tm && k.tn == t.tn && k.bh == t.bh && k.ks == t.ks && k.nr == t.nr &&
        k.nw == t.nw && k.pf == (int)t.pf && k.bf == bf && k.lds == lds)
      return k.n;
  }
  WGrad3 p{};
  g_w3probe = W3Probe{};
  g_w3probe.on = true;
  if (t.bh == 8) wgrad3_launch<8>(p, t, dim3(1), lds, nullptr);
  else wgrad3_launch<4>(p, t, dim3(1), lds, nullptr);
  g_w3probe.on = false;
  int n = 0;
  if (!g_w3probe.fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(
                           &n, g_w3probe.fn, (int)g_w3probe.threads, lds) != hipSuccess ||
      n < 1) {
    (void)hipGetLastError();
    n = 1;
  }
  if (ncache < 32) cache[ncache++] = Key{t.tm, t.tn, t.bh, t.ks, t.nr, t.nw, (int)t.pf, bf, lds, n};
  return n;
}
#endif  // VAE2_PART(3)

extern "C" {

#if VAE2_PART(0)
int64_t vae2_conv2d_packed_size(int64_t cout, int64_t cin, int k, int mode) {
  int rows = mode == 0 ? round_up((int)cout, 64) : round_up((int)cin, 64);
  int cols4 = mode == 0 ? round_up((int)cin, 4) : round_up((int)cout, 4);
  return (int64_t)rows * k * k * cols4;
}

int vae2_conv2d_pack_weight_ld(const float* w, int64_t cout, int64_t cin, int k, int mode,
                               int64_t ld, float* out, void* stream) {
  const char* fn = "vae2_conv2d_pack_weight";
  VAE2_REQUIRE(w && out && cout > 0 && cin > 0 && k > 0 && (mode == 0 || mode == 1), fn,
               "bad arguments");
  VAE2_REQUIRE(ld >= cin * k * k && ld < (int64_t(1) << 31), fn, "bad row stride");
  int64_t total = vae2_conv2d_packed_size(cout, cin, k, mode);
  VAE2_LAUNCH(pack_weight_kernel, dim3(ew_blocks(total, 256, 2048)), dim3(256), 0,
                     as_stream(stream), w, (int)cout, (int)cin, k * k, mode, (int)ld, out);
  return check_launch(fn);
}

int vae2_conv2d_pack_weight(const float* w, int64_t cout, int64_t cin, int k, int mode,
                            float* out, void* stream) {
  return vae2_conv2d_pack_weight_ld(w, cout, cin, k, mode, cin * k * k, out, stream);
}

int vae2_conv2d_pack_weights(const vae2_pack_job* jobs, int64_t njobs, void* stream) {
  const char* fn = "vae2_conv2d_pack_weights";
  VAE2_REQUIRE(jobs && njobs > 0 && njobs <= 65535, fn, "bad job table");
  VAE2_LAUNCH(pack_weights_batched_kernel, dim3(32, (unsigned)njobs), dim3(256), 0,
                     as_stream(stream), jobs);
  return check_launch(fn);
}

// Launch-shape tuning knobs (A/B measurements; every setting computes the same result):
// key 0 = igemm minimum workgroups (0: the default row-tile rule); key 4 = gemm1x1 N tiles
// per workgroup (3..8).  Returns the previous
// value, or -1 for an unknown key.
int vae2_conv2d_set_tune(int key, int value) {
  if (key == 0) {
    const int prev = g_igemm_minblk;
    g_igemm_minblk = value < 0 ? 0 : value;
    return prev;
  }
  if (key == 1) {
    const int prev = g_wgrad_cols;
    g_wgrad_cols = value ? 1 : 0;
    return prev;
  }
  if (key == 2) {
    const int prev = g_dconv_nw8;
    g_dconv_nw8 = value ? 1 : 0;
    return prev;
  }
  if (key == 3) {
    const int prev = g_wgrad_nw8;
    g_wgrad_nw8 = value ? 1 : 0;
    return prev;
  }
  if (key == 4) {
    if (value < 3 || value > 8) return -1;  // rejected, setting unchanged
    const int prev = g_gemm1_tn;
    g_gemm1_tn = value;
    return prev;
  }
  if (key == 5) {
    const int prev = g_gemm1_tm;
    g_gemm1_tm = value == 1 ? 1 : 2;
    return prev;
  }
  if (key == 6) {
    if (value < 0 || value > 2) return -1;
    const int prev = g_igemm_nr;
    g_igemm_nr = value;
    return prev;
  }
  if (key == 8) {  // bn.hip: buffer-resource BatchNorm bodies
    const int prev = g_bn_v2;
    g_bn_v2 = value ? 1 : 0;
    return prev;
  }
  if (key == 7) {
    if (value < 0 || value > 3) return -1;
    const int prev = g_wgrad_narrow;
    g_wgrad_narrow = value;
    return prev;
  }
  if (key == 9) {  // dconv_stream.hip: streaming direct 3x3 for 18 / 36 channels
    const int prev = g_dconv_stream;
    g_dconv_stream = value >= 0 && value <= 3 ? value : 3;
    return prev;
  }
  if (key == 18) {  // gather weight gradient: target workgroups (split count)
    if (value < 256 || value > 8192) return -1;
    const int prev = g_wgrad_wgs;
    g_wgrad_wgs = value;
    return prev;
  }
  if (key == 21) {  // resample.hip: the fuse sum a channel quad per thread (1) or per channel
    const int prev = g_fuse_quad;
    g_fuse_quad = value ? 1 : 0;
    return prev;
  }
  if (key == 20) {  // bn.hip: apply kernels' resident-block budget (0 = one block per chunk)
    if (value < 0 || value > 65536) return -1;
    const int prev = g_bn_apply_res;
    g_bn_apply_res = value;
    return prev;
  }
  if (key == 19) {  // bn.hip: BatchNorm blocks per layer (at most)
    if (value < 256 || value > 8192) return -1;
    const int prev = g_bn_blocks;
    g_bn_blocks = value;
    return prev;
  }
  if (key == 16) {  // wgrad_narrow.hip: minimum tiles per split (partial slab)
    if (value < 1 || value > 2) return -1;
    const int prev = g_wgrad_narrow_tps;
    g_wgrad_narrow_tps = value;
    return prev;
  }
  if (key == 17) {  // dconv_stream.hip: minimum 4-row steps per band
    if (value < 1 || value > 2) return -1;
    const int prev = g_dconv_stream_spb;
    g_dconv_stream_spb = value;
    return prev;
  }
  if (key == 15) {  // direct 3x3: K split for layers short of workgroups (0, 1: 2, 2: 4 shares)
    if (value < 0 || value > 2) return -1;
    const int prev = g_dconv_ksp;
    g_dconv_ksp = value;
    return prev;
  }
  if (key == 14) {  // direct 3x3: 72 channels as two 32 + 4 N blocks
    const int prev = g_dconv_split72;
    g_dconv_split72 = value ? 1 : 0;
    return prev;
  }
  if (key == 13) {  // direct 3x3: 16-channel N blocks for layers short of workgroups
    const int prev = g_dconv_n16;
    g_dconv_n16 = value ? 1 : 0;
    return prev;
  }
  if (key == 12) {  // gather GEMM: K-step table (1) or per-chunk tap arithmetic (0)
    const int prev = g_igemm_tab;
    g_igemm_tab = value ? 1 : 0;
    return prev;
  }
  if (key == 11) {  // dconv_stream.hip: 18-channel weights in LDS (B operand) or global
    const int prev = g_dconv_stream_bl;
    g_dconv_stream_bl = value ? 1 : 0;
    return prev;
  }
  if (key == 10) {  // dconv_stream.hip: target workgroups per CU (0 = auto)
    const int prev = g_dconv_stream_wpc;
    g_dconv_stream_wpc = value >= 0 && value <= 8 ? value : 0;
    return prev;
  }
  return -1;
}

int vae2_conv2d_set_mfma_bf16(int on) {
  const int prev = g_bf16;
  g_bf16 = on ? 1 : 0;
  return prev;
}

#endif  // VAE2_PART(0)

#if VAE2_PART(3)
int vae2_wgrad_defer(int on) {
  const int prev = g_wr_defer ? 1 : 0;
  g_wr_defer = on != 0;
  return prev;
}

static int wgrad_flush_impl(void* stream, bool own_only) {
  const char* fn = "vae2_wgrad_flush";
  hipStream_t want = as_stream(stream);
  std::vector<WRQueued> q;
  {
    std::lock_guard<std::mutex> lk(g_wr_mu);
    if (own_only) {  // only the jobs queued from this stream (no cross-stream ordering)
      std::vector<WRQueued> keep;
      for (const WRQueued& j : g_wr_queue) (j.stream == want ? q : keep).push_back(j);
      g_wr_queue.swap(keep);
    } else {
      q.swap(g_wr_queue);
    }
  }
  size_t i = 0;
  // every job on the given stream: the caller orders it after the jobs' own streams
  while (i < q.size()) {  // kWrMaxJobs per launch
    WRMulti m{};
    hipStream_t st = want;
    int blocks = 0;
    while (i < q.size() && m.n < kWrMaxJobs) {
      WRJob j = q[i].job;
      // a job accumulating into dW elements a job of this launch writes waits for the
      // next launch (e.g. a discriminator applied to real and fake inputs)
      const float* lo = j.dw;
      const float* hi = j.dw + (int64_t)(j.cout - 1) * j.ld + (int64_t)j.cin * j.k * j.k;
      bool clash = false;
      for (int u = 0; u < m.n; ++u) {
        const float* lo2 = m.j[u].dw;
        const float* hi2 = m.j[u].dw + (int64_t)(m.j[u].cout - 1) * m.j[u].ld +
                           (int64_t)m.j[u].cin * m.j[u].k * m.j[u].k;
        if (lo < hi2 && lo2 < hi) clash = true;
      }
      if (clash) break;
      j.blk0 = blocks;
      blocks += (int)ceil_div((int64_t)j.cout * j.k * j.k * j.cin4, 32);
      m.j[m.n++] = j;
      ++i;
    }
    VAE2_LAUNCH(wgrad_reduce_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, st, m);
    const int rc = check_launch(fn);
    if (rc) return rc;
  }
  return 0;
}

int vae2_wgrad_flush(void* stream) { return wgrad_flush_impl(stream, false); }

int vae2_wgrad_flush_stream(void* stream) { return wgrad_flush_impl(stream, true); }



#endif  // VAE2_PART(3)

#if VAE2_PART(0)
int vae2_conv2d_set_algo(int algo) {
  const int prev = g_conv_algo + (g_wide_tiles ? 0 : 4) + (g_ksplit ? 0 : 8) +
                   (g_dconv_nr ? 0 : 16) + (g_gemm1 ? 0 : 32) + (g_vec_out ? 0 : 64) +
                   (g_dconv_nr_wide ? 0 : 128);
  const int a = algo & 7;
  if (algo >= 0 && algo <= 255 && a <= 6 && a != 3) {
    g_dconv_nr_wide = (algo & 128) ? 0 : 1;
    g_conv_algo = a & 3;
    g_wide_tiles = a < 4;
    g_ksplit = !(algo & 8);
    g_dconv_nr = !(algo & 16);
    g_gemm1 = !(algo & 32);
    g_vec_out = !(algo & 64);
  }
  return prev;
}

int64_t vae2_conv2d_fwd_stats_rows(const float* x, const vae2_act* xd, const vae2_act* yd,
                                   int k, int stride, int pad) {
  if (!act_ok(xd) || !act_ok(yd)) return 0;
  if (dconv_use(xd, yd, k, stride, pad, x)) return dconv_rows(xd, yd);
  G1Tile g1;
  if (gemm1_pick(xd, yd, k, stride, pad, x, &g1)) return g1.grid_x;
  return igemm_rows(act_pixels(yd), (int)yd->c, k * k, round_up((int)xd->c, 4));
}

int vae2_conv2d_fwd_kernel_name(const vae2_act* xd, const vae2_act* yd, int k, int stride,
                                int pad, char* buf, int64_t len) {
  if (!xd || !yd || !buf || len <= 0) return -22;
  if (dconv_use(xd, yd, k, stride, pad, (const float*)16)) {
    if (stream_use(xd, yd)) {
      const int q = (int)((xd->c + 3) / 4);
      snprintf(buf, (size_t)len, "dconv3s_kernel<%d, %d, %d, false", q == 5 ? 1 : 2,
               q == 5 ? 2 : 4, q);
      return 0;
    }
    DTile d = pick_dtile(xd, yd);
    if (d.nr)
      snprintf(buf, (size_t)len, "dconv3_kernel<%d, %d, false, false, %d>", d.tm, d.tn, d.nr);
    else
      snprintf(buf, (size_t)len, "dconv3_kernel<%d, %d, false>", d.tm, d.tn);
    return 0;
  }
  G1Tile g1;
  if (gemm1_pick(xd, yd, k, stride, pad, (const float*)16, &g1)) {
    snprintf(buf, (size_t)len, "gemm1x1_kernel<%d, %d>", g1.tm, g1.tn);
    return 0;
  }
  Tile t = pick_igemm_tile(act_pixels(yd), (int)yd->c, k * k, round_up((int)xd->c, 4), 1);
  if (t.ks > 1)
    snprintf(buf, (size_t)len, "igemm_kernel<%d, %d, true, 0, %d>", t.tm, t.tn, t.ks);
  else
    snprintf(buf, (size_t)len, "igemm_kernel<%d, %d, true, 0>", t.tm, t.tn);
  return 0;
}

int vae2_conv2d_fwd(const float* x, const vae2_act* xd, const float* wp,
                    const float* bias, float* y, const vae2_act* yd, int k,
                    int stride, int pad, float beta, float* stats,
                    void* stream) {
  const char* fn = "vae2_conv2d_fwd";
  VAE2_REQUIRE(x && wp && y, fn, "null pointer");
  VAE2_REQUIRE(conv_shapes_ok(xd, yd, k, stride, pad), fn, "inconsistent conv shapes");
  VAE2_REQUIRE(fits32(xd) && fits32(yd), fn, "tensor too large for 32-bit indexing");
  if (dconv_use(xd, yd, k, stride, pad, x)) {
    return launch_dconv(x, xd, wp, (uint32_t)(vae2_conv2d_packed_size(yd->c, xd->c, k, 0) * 4),
                        bias, y, yd, beta, stats, false, as_stream(stream), fn);
  }
  G1Tile g1;
  if (gemm1_pick(xd, yd, k, stride, pad, x, &g1)) {
    const int rc = launch_gemm1(x, xd, wp,
                                (uint32_t)(vae2_conv2d_packed_size(yd->c, xd->c, k, 0) * 4),
                                bias, y, yd, beta, stats, g1, as_stream(stream), fn);
    if (rc != -1) return rc;
    VAE2_REQUIRE(stats == nullptr, fn, "BN statistics need a 16-byte aligned output here");
  }
  IGemm p{};
  p.a = x; p.a_ps = (int)xd->ps; p.a_c = (int)xd->c; p.a_c4 = round_up((int)xd->c, 4);
  p.a_h = (int)xd->h; p.a_w = (int)xd->w;
  p.g_n = (int)yd->n; p.g_h = (int)yd->h; p.g_w = (int)yd->w;
  p.a_step = stride;
  p.nth = k; p.ntw = k;
  p.dh0 = -pad; p.dhs = 1; p.dw0 = -pad; p.dws = 1;
  p.kh0 = 0; p.khs = 1; p.kw0 = 0; p.kws = 1; p.ksz = k;
  p.w = wp; p.n = (int)yd->c;
  p.a_bytes = act_bytes(xd);
  p.w_bytes = (uint32_t)(vae2_conv2d_packed_size(yd->c, xd->c, k, 0) * 4);
  p.bias = bias;
  p.y = y; p.y_ps = (int)yd->ps; p.y_h = (int)yd->h; p.y_w = (int)yd->w;
  p.y_step = 1; p.y_offh = 0; p.y_offw = 0;
  p.beta = beta;
  p.stats = stats;
  return launch_igemm(p, 0, as_stream(stream), fn);
}

int vae2_conv2d_bnin_ok(const float* x, const vae2_act* xd, const vae2_act* yd, int k,
                        int stride, int pad) {
  if (!x || !conv_shapes_ok(xd, yd, k, stride, pad) || !fits32(xd) || !fits32(yd)) return 0;
  return !g_bf16 && dconv_use(xd, yd, k, stride, pad, x) && g_conv_algo != 1 &&
         wgrad3_shape_ok(xd, yd, k, stride, pad) && vec_ok(x, (int)xd->ps);
}

int vae2_conv2d_fwd_bnin(const float* x, const vae2_act* xd, const float* bn_save, int relu,
                         const float* wp, const float* bias, float* y, const vae2_act* yd,
                         int k, int stride, int pad, float beta, float* stats, void* stream) {
  const char* fn = "vae2_conv2d_fwd_bnin";
  VAE2_REQUIRE(x && wp && y && bn_save, fn, "null pointer");
  VAE2_REQUIRE(conv_shapes_ok(xd, yd, k, stride, pad), fn, "inconsistent conv shapes");
  VAE2_REQUIRE(vae2_conv2d_bnin_ok(x, xd, yd, k, stride, pad), fn,
               "input BatchNorm needs the direct 3x3 kernels (vae2_conv2d_bnin_ok)");
  BnSide bn;
  bn.isave = bn_save;
  bn.irelu = relu ? 1 : 0;
  return launch_dconv(x, xd, wp, (uint32_t)(vae2_conv2d_packed_size(yd->c, xd->c, k, 0) * 4),
                      bias, y, yd, beta, stats, false, as_stream(stream), fn, bn);
}

static int igemm_dgrad_setup(IGemm& p, const float* dy, const vae2_act* dyd, const float* wp,
                             float* dx, const vae2_act* dxd, int k, int stride, int pad,
                             float beta);
static int64_t igemm_dgrad_rows(const float* dy, const vae2_act* dyd, const vae2_act* dxd,
                                int k, int stride, int pad);

// Round 6: every data-gradient kernel family writes the partials -- the direct 3x3 kernels
// (round 3), the persistent 1x1 GEMM and the gather kernel (every other conv, incl. the
// stride-2 classes) -- so the rows follow vae2_conv2d_bwd_data's own dispatch.
int64_t vae2_conv2d_bwd_data_bnpart_rows(const float* dy, const vae2_act* dyd,
                                         const vae2_act* dxd, int k, int stride, int pad) {
  if (!dy || !conv_shapes_ok(dxd, dyd, k, stride, pad) || !fits32(dxd) || !fits32(dyd))
    return 0;
  if (g_bf16) return 0;
  if (dconv_use(dyd, dxd, k, stride, pad, dy)) return dconv_rows(dyd, dxd);
  G1Tile g1;
  if (gemm1_pick(dyd, dxd, k, stride, pad, dy, &g1)) return g1.grid_x;
  return igemm_dgrad_rows(dy, dyd, dxd, k, stride, pad);
}

int vae2_conv2d_bwd_data_bnpart(const float* dy, const vae2_act* dyd, const float* wp,
                                float* dx, const vae2_act* dxd, int k, int stride, int pad,
                                const float* bn_x, const vae2_act* bn_xd, const float* bn_save,
                                int relu, float* partials, void* stream) {
  const char* fn = "vae2_conv2d_bwd_data_bnpart";
  VAE2_REQUIRE(dy && wp && dx && bn_x && bn_xd && bn_save && partials, fn, "null pointer");
  VAE2_REQUIRE(conv_shapes_ok(dxd, dyd, k, stride, pad), fn, "inconsistent conv shapes");
  VAE2_REQUIRE(bn_xd->n == dxd->n && bn_xd->h == dxd->h && bn_xd->w == dxd->w &&
               bn_xd->c == dxd->c && bn_xd->ps >= bn_xd->c && fits32(bn_xd), fn,
               "BatchNorm input shape must match dx");
  VAE2_REQUIRE(vae2_conv2d_bwd_data_bnpart_rows(dy, dyd, dxd, k, stride, pad) > 0, fn,
               "BatchNorm partials are not available for this geometry "
               "(vae2_conv2d_bwd_data_bnpart_rows)");
  const uint32_t wbytes = (uint32_t)(vae2_conv2d_packed_size(dyd->c, dxd->c, k, 1) * 4);
  if (dconv_use(dyd, dxd, k, stride, pad, dy)) {
    BnSide bn;
    bn.bx = bn_x;
    bn.bx_ps = (int)bn_xd->ps;
    bn.bx_bytes = act_bytes(bn_xd);
    bn.bsave = bn_save;
    bn.brelu = relu ? 1 : 0;
    return launch_dconv(dy, dyd, wp, wbytes, nullptr, dx, dxd, 0.f, partials, true,
                        as_stream(stream), fn, bn);
  }
  G1Tile g1;
  if (gemm1_pick(dyd, dxd, k, stride, pad, dy, &g1)) {
    const int rc = launch_gemm1(dy, dyd, wp, wbytes, nullptr, dx, dxd, 0.f, partials, g1,
                                as_stream(stream), fn, bn_x, (int)bn_xd->ps, relu ? 1 : 0,
                                bn_save, act_bytes(bn_xd));
    VAE2_REQUIRE(rc != -1, fn, "1x1 GEMM refused the partials form");
    return rc;
  }
  IGemm p{};
  const int ncls = igemm_dgrad_setup(p, dy, dyd, wp, dx, dxd, k, stride, pad, 0.f);
  VAE2_REQUIRE(ncls > 0, fn, "stride > 2 is not supported");
  p.stats = partials;
  p.bx = bn_x;
  p.bx_ps = (int)bn_xd->ps;
  p.bx_bytes = act_bytes(bn_xd);
  p.bsave = bn_save;
  p.brelu = relu ? 1 : 0;
  return launch_igemm(p, 1, as_stream(stream), fn, ncls);
}

int vae2_conv2d_bwd_data(const float* dy, const vae2_act* dyd, const float* wp,
                         float* dx, const vae2_act* dxd, int k, int stride,
                         int pad, float beta, void* stream) {
  const char* fn = "vae2_conv2d_bwd_data";
  VAE2_REQUIRE(dy && wp && dx, fn, "null pointer");
  VAE2_REQUIRE(conv_shapes_ok(dxd, dyd, k, stride, pad), fn, "inconsistent conv shapes");
  VAE2_REQUIRE(fits32(dxd) && fits32(dyd), fn, "tensor too large for 32-bit indexing");
  if (dconv_use(dyd, dxd, k, stride, pad, dy))
    return launch_dconv(dy, dyd, wp, (uint32_t)(vae2_conv2d_packed_size(dyd->c, dxd->c, k, 1) * 4),
                        nullptr, dx, dxd, beta, nullptr, true, as_stream(stream), fn);
  G1Tile g1;
  if (gemm1_pick(dyd, dxd, k, stride, pad, dy, &g1)) {
    const int rc = launch_gemm1(dy, dyd, wp,
                                (uint32_t)(vae2_conv2d_packed_size(dyd->c, dxd->c, k, 1) * 4),
                                nullptr, dx, dxd, beta, nullptr, g1, as_stream(stream), fn);
    if (rc != -1) return rc;
  }
  IGemm p{};
  const int ncls = igemm_dgrad_setup(p, dy, dyd, wp, dx, dxd, k, stride, pad, beta);
  VAE2_REQUIRE(ncls >= 0, fn, "stride > 2 is not supported");
  if (ncls == 0) return 0;
  return launch_igemm(p, 1, as_stream(stream), fn, ncls);
}

// The gather kernel's data-gradient setup (vae2_conv2d_bwd_data, the _bnpart form and its
// rows query): returns the number of stride-parity classes (0: nothing to do, -1: stride > 2).
static int igemm_dgrad_setup(IGemm& p, const float* dy, const vae2_act* dyd, const float* wp,
                             float* dx, const vae2_act* dxd, int k, int stride, int pad,
                             float beta) {
  // Stride-parity classes (ph, pw) of the input pixels: input row ih = stride*i + ph
  // receives from output row oh = (ih + pad - kh)/stride for every kh with
  // (ph + pad - kh) % stride == 0.  All classes run in one launch (class = blockIdx.z);
  // each has only its valid taps.
  p.a = dy; p.a_ps = (int)dyd->ps; p.a_c = (int)dyd->c; p.a_c4 = round_up((int)dyd->c, 4);
  p.a_h = (int)dyd->h; p.a_w = (int)dyd->w;
  p.g_n = (int)dxd->n;
  p.a_step = 1;
  p.dhs = -1; p.dws = -1;
  p.khs = stride; p.kws = stride; p.ksz = k;
  p.w = wp; p.n = (int)dxd->c;
  p.a_bytes = act_bytes(dyd);
  p.w_bytes = (uint32_t)(vae2_conv2d_packed_size(dyd->c, dxd->c, k, 1) * 4);
  p.bias = nullptr;
  p.y = dx; p.y_ps = (int)dxd->ps; p.y_h = (int)dxd->h; p.y_w = (int)dxd->w;
  p.y_step = stride;
  p.beta = beta;
  p.stats = nullptr;
  int ncls = 0;
  for (int ph = 0; ph < stride; ++ph) {
    for (int pw = 0; pw < stride; ++pw) {
      int gh = (int)((dxd->h - ph + stride - 1) / stride);
      int gw = (int)((dxd->w - pw + stride - 1) / stride);
      if (gh <= 0 || gw <= 0) continue;
      if (ncls >= 4) return -1;
      int kh0 = ((ph + pad) % stride + stride) % stride;
      int kw0 = ((pw + pad) % stride + stride) % stride;
      int nth = kh0 < k ? (k - 1 - kh0) / stride + 1 : 0;
      int ntw = kw0 < k ? (k - 1 - kw0) / stride + 1 : 0;
      IGemm::Cls& c = p.cls[ncls++];
      c.g_h = gh; c.g_w = gw;
      c.nth = nth; c.ntw = ntw;
      c.dh0 = (ph + pad - kh0) / stride;
      c.dw0 = (pw + pad - kw0) / stride;
      c.kh0 = kh0; c.kw0 = kw0;
      c.y_offh = ph; c.y_offw = pw;
      if (nth == 0 || ntw == 0) { c.nth = 0; c.ntw = 1; }
    }
  }
  if (ncls == 0) return 0;
  {
    const IGemm::Cls& c = p.cls[0];  // the single-class launch reads the plain fields
    p.g_h = c.g_h; p.g_w = c.g_w; p.nth = c.nth; p.ntw = c.ntw;
    p.dh0 = c.dh0; p.dw0 = c.dw0; p.kh0 = c.kh0; p.kw0 = c.kw0;
    p.y_offh = c.y_offh; p.y_offw = c.y_offw;
  }
  return ncls;
}

// Partial-statistics rows of a gather-kernel data gradient (gridDim.x * classes).
static int64_t igemm_dgrad_rows(const float* dy, const vae2_act* dyd, const vae2_act* dxd,
                                int k, int stride, int pad) {
  IGemm p{};
  const int ncls = igemm_dgrad_setup(p, dy, dyd, nullptr, nullptr, dxd, k, stride, pad, 0.f);
  if (ncls <= 0) return 0;
  int64_t M = (int64_t)p.g_n * p.g_h * p.g_w;
  int max_taps = p.nth * p.ntw;
  for (int c = 0; c < ncls && ncls > 1; ++c) {
    const IGemm::Cls& q = p.cls[c];
    const int64_t mc = (int64_t)p.g_n * q.g_h * q.g_w;
    if (mc > M) M = mc;
    if (q.nth * q.ntw > max_taps) max_taps = q.nth * q.ntw;
  }
  const Tile t = pick_igemm_tile(M, p.n, max_taps, p.a_c4, ncls);
  return ceil_div(M, igemm_rows_per_block(t)) * ncls;
}

#endif  // VAE2_PART(0)

#if VAE2_PART(2)
// Independent convolutions in one call (one HRNet depth level): the jobs the direct 3x3
// kernel takes are launched together, up to kDcGroup per launch, grouped by tile shape
// and direction (jobs writing the same output never share a launch); the others go
// through vae2_conv2d_fwd / vae2_conv2d_bwd_data one by one.
static int g_conv_group = 0;  // measured slower in the full step: off by default

int vae2_conv2d_set_grouping(int on) {
  const int prev = g_conv_group;
  g_conv_group = on ? 1 : 0;
  return prev;
}

int vae2_conv2d_multi(int n, const vae2_conv_job* jobs, void* stream) {
  const char* fn = "vae2_conv2d_multi";
  VAE2_REQUIRE(n >= 0 && (n == 0 || jobs), fn, "bad arguments");
  hipStream_t s = as_stream(stream);
  struct Bucket {
    int tm, tn, flip, cnt, tot;
    DConvGroup g;
    size_t shm;
    const float* outs[kDcGroup];
  };
  Bucket b[8];
  int nb = 0;
  auto flush = [&](Bucket& k) -> int {
    if (k.cnt == 0) return 0;
    k.g.n = k.cnt;
    k.g.start[k.cnt] = k.tot;
    for (int q = k.cnt; q < kDcGroup; ++q) { k.g.start[q + 1] = k.tot; k.g.tiles[q] = 1; }
    const dim3 grid((unsigned)k.tot);
    if (k.tm == 4) {
      if (k.flip) dconv_group_launch_tn<4, true>(k.g, k.tn, grid, k.shm, s);
      else dconv_group_launch_tn<4, false>(k.g, k.tn, grid, k.shm, s);
    } else {
      if (k.flip) dconv_group_launch_tn<2, true>(k.g, k.tn, grid, k.shm, s);
      else dconv_group_launch_tn<2, false>(k.g, k.tn, grid, k.shm, s);
    }
    k.cnt = 0; k.tot = 0; k.shm = 0;
    return check_launch(fn);
  };
  // a job writing an output some queued job also writes runs after that job's launch
  auto flush_holding = [&](const float* out) -> int {
    for (int k = 0; k < nb; ++k)
      for (int q = 0; q < b[k].cnt; ++q)
        if (b[k].outs[q] == out) return flush(b[k]);
    return 0;
  };
  for (int i = 0; i < n; ++i) {
    const vae2_conv_job& J = jobs[i];
    VAE2_REQUIRE(J.kind == 0 || J.kind == 1, fn, "job kind must be 0 (forward) or 1 (data grad)");
    if (int rc = flush_holding(J.y)) return rc;
    const bool fwd = J.kind == 0;
    const vae2_act* ad = &J.xd;  // the kernel's input: x (forward) or dy (data gradient)
    const vae2_act* od = &J.yd;
    bool direct = g_conv_group && J.x && J.wp && J.y &&
                  (fwd ? conv_shapes_ok(ad, od, J.k, J.stride, J.pad)
                       : conv_shapes_ok(od, ad, J.k, J.stride, J.pad)) &&
                  fits32(ad) && fits32(od) && dconv_use(ad, od, J.k, J.stride, J.pad, J.x) &&
                  !stream_use(ad, od) &&         // (streaming layers: their own launch)
                  pick_dtile(ad, od).nr == 0 &&  // (remainder layers: their own launch)
                  pick_dtile(ad, od).nw == 4;    // (8-wave tiles: their own launch)
    if (!direct) {
      int rc = fwd ? vae2_conv2d_fwd(J.x, ad, J.wp, J.bias, J.y, od, J.k, J.stride, J.pad,
                                     J.beta, J.stats, stream)
                   : vae2_conv2d_bwd_data(J.x, ad, J.wp, J.y, od, J.k, J.stride, J.pad,
                                          J.beta, stream);
      if (rc) return rc;
      continue;
    }
    const DTile d = pick_dtile(ad, od, false);
    const uint32_t wb = (uint32_t)((fwd ? vae2_conv2d_packed_size(od->c, ad->c, J.k, 0)
                                        : vae2_conv2d_packed_size(ad->c, od->c, J.k, 1)) * 4);
    int k = 0;
    while (k < nb && !(b[k].tm == d.tm && b[k].tn == d.tn && b[k].flip == (fwd ? 0 : 1))) ++k;
    if (k == nb) {
      VAE2_REQUIRE(nb < 8, fn, "too many tile shapes");
      b[nb] = Bucket{};
      b[nb].tm = d.tm; b[nb].tn = d.tn; b[nb].flip = fwd ? 0 : 1;
      ++nb;
    }
    Bucket& B = b[k];
    if (B.cnt == kDcGroup) {
      int rc = flush(B);
      if (rc) return rc;
    }
    const int tiles = (int)(ad->n * d.tiles_h * d.tiles_w);
    B.g.p[B.cnt] = make_dconv(d, J.x, ad, J.wp, wb, fwd ? J.bias : nullptr, J.y, od, J.beta,
                              fwd ? J.stats : nullptr);
    B.g.start[B.cnt] = B.tot;
    B.g.tiles[B.cnt] = tiles;
    B.outs[B.cnt] = J.y;
    B.tot += tiles * d.nblk;
    const size_t sh = dconv_shm(d);
    if (sh > B.shm) B.shm = sh;
    ++B.cnt;
  }
  for (int k = 0; k < nb; ++k) {
    int rc = flush(b[k]);
    if (rc) return rc;
  }
  return 0;
}

#endif  // VAE2_PART(2)

#if VAE2_PART(3)
int64_t vae2_conv2d_bwd_weight_ws_size(const vae2_act* xd, const vae2_act* dyd, int k) {
  if (!act_ok(xd) || !act_ok(dyd)) return 0;
  int ncol4 = k * k * round_up((int)xd->c, 4);
  WTile t = pick_wtile(act_pixels(dyd), (int)dyd->c, ncol4);
  int64_t part = (int64_t)t.splits * dyd->c * ncol4;
  if ((k == 3 || k == 1) && xd->h == dyd->h && xd->w == dyd->w) {  // direct kernel may run
    W3Tile t3 = pick_w3tile(xd, dyd, k);
    const int64_t part3 = (int64_t)t3.splits * dyd->c * ncol4;
    if (part3 > part) part = part3;
    const int64_t partn = wgrad3n_splits(xd, dyd) * dyd->c * ncol4;
    if (partn > part) part = partn;
  }
  int64_t bias_part = 2 * vae2_bn_partial_rows(dyd) * dyd->c;
  return part + bias_part + 4;
}

static int bwd_weight_impl(const float* x, const vae2_act* xd, const float* dy,
                           const vae2_act* dyd, float* dw, int64_t dw_ld, float* dbias,
                           int k, int stride, int pad, int accumulate, float* ws,
                           int64_t ws_size, void* stream, const float* isave, int irelu,
                           const char* fn) {
  VAE2_REQUIRE(xd && dw_ld >= xd->c * k * k, fn, "bad dW row stride");
  VAE2_REQUIRE(x && dy && dw && ws, fn, "null pointer");
  VAE2_REQUIRE(conv_shapes_ok(xd, dyd, k, stride, pad), fn, "inconsistent conv shapes");
  VAE2_REQUIRE(fits32(xd) && fits32(dyd), fn, "tensor too large for 32-bit indexing");
  VAE2_REQUIRE(ws_size >= vae2_conv2d_bwd_weight_ws_size(xd, dyd, k), fn, "workspace too small");
  hipStream_t s = as_stream(stream);
  const int cin4 = round_up((int)xd->c, 4);
  const int ncol4 = k * k * cin4;
  int splits = 0;
  const bool direct = g_conv_algo != 1 && wgrad3_shape_ok(xd, dyd, k, stride, pad) &&
                      vec_ok(x, (int)xd->ps) && vec_ok(dy, (int)dyd->ps);
  VAE2_REQUIRE(direct || !isave, fn,
               "input BatchNorm needs the direct 3x3 weight-gradient kernel (vae2_conv2d_bnin_ok)");
  if (direct && k == 3) {  // the 18 / 36 / 72-channel branches (wgrad_narrow.hip)
    splits = wgrad3n_launch(x, xd, dy, dyd, ws, isave, irelu, act_bytes(xd), act_bytes(dyd), s);
    if (splits < 0) return check_launch(fn);
  }
  if (direct && !splits) {
    W3Tile t3 = pick_w3tile(xd, dyd, k);
    WGrad3 q{};
    q.x = x; q.x_ps = (int)xd->ps; q.cin = (int)xd->c; q.cin4 = cin4;
    q.h = (int)xd->h; q.w = (int)xd->w;
    q.dy = dy; q.dy_ps = (int)dyd->ps; q.cout = (int)dyd->c;
    q.tiles_h = t3.tiles_h; q.tiles_w = t3.tiles_w; q.ntiles = t3.ntiles;
    q.tiles_per_split = t3.tps;
    q.csw = t3.csw; q.n_ci_slabs = t3.n_ci_slabs;
    q.x_bytes = act_bytes(xd); q.dy_bytes = act_bytes(dyd);
    q.part = ws;
    q.isave = isave;
    q.irelu = irelu ? 1 : 0;
    dim3 grid((unsigned)t3.splits, (unsigned)(t3.n_ci_slabs * t3.n_co_slabs));
    const size_t shm = wgrad3_lds(t3);
    if (t3.bh == 8) wgrad3_launch<8>(q, t3, grid, shm, s);
    else wgrad3_launch<4>(q, t3, grid, shm, s);
    int rc = check_launch(fn);
    if (rc) return rc;
    splits = t3.splits;
  }
  WTile t = pick_wtile(act_pixels(dyd), (int)dyd->c, ncol4);
  if (splits) goto reduce;
  {
  WGrad p{};
  p.x = x; p.x_ps = (int)xd->ps; p.cin = (int)xd->c; p.cin4 = cin4;
  p.x_h = (int)xd->h; p.x_w = (int)xd->w;
  p.dy = dy; p.dy_ps = (int)dyd->ps; p.cout = (int)dyd->c;
  p.o_n = (int)dyd->n; p.o_h = (int)dyd->h; p.o_w = (int)dyd->w;
  p.k = k; p.stride = stride; p.pad = pad;
  p.P = (int)act_pixels(dyd);
  p.px_split = t.px_split;
  p.part = ws;
  p.x_bytes = act_bytes(xd);
  p.dy_bytes = act_bytes(dyd);
  p.ohw_div = FastDiv((uint32_t)(dyd->h * dyd->w));
  p.ow_div = FastDiv((uint32_t)dyd->w);
  p.cin4_div = FastDiv((uint32_t)cin4);
  dim3 grid(t.gx, t.gy, (unsigned)t.splits);
  // 16-byte channel-quad operand loads (quad-transposed into fragments)
  const bool v4 = g_vec_out && vec_ok(x, (int)xd->ps) && vec_ok(dy, (int)dyd->ps);
  switch (t.tm) {
    case 1: launch_wgrad_tn<1>(p, t.tn, grid, s, v4); break;
    case 2: launch_wgrad_tn<2>(p, t.tn, grid, s, v4); break;
    case 3: launch_wgrad_tn<3>(p, t.tn, grid, s, v4); break;
    default: launch_wgrad_tn<4>(p, t.tn, grid, s, v4); break;
  }
  int rc = check_launch(fn);
  if (rc) return rc;
  splits = t.splits;
  }
reduce:
  int64_t slab = dyd->c * (int64_t)ncol4;
  int rc = 0;
  if (g_wr_defer) {
    WRJob j{ws, dw, dw_ld, splits, (int)dyd->c, (int)xd->c, cin4, k, accumulate, 0};
    std::lock_guard<std::mutex> lk(g_wr_mu);
    g_wr_queue.push_back(WRQueued{j, s});
  } else {
    VAE2_LAUNCH(wgrad_reduce_kernel, dim3((unsigned)ceil_div(slab, 32)), dim3(256), 0, s,
                (const float*)ws, splits, (int)dyd->c, (int)xd->c, cin4, k, dw, dw_ld,
                accumulate);
    rc = check_launch(fn);
    if (rc) return rc;
  }
  if (dbias) {
    // bias partial rows live after the largest partial-slab area the workspace holds
    const int64_t part_max = vae2_conv2d_bwd_weight_ws_size(xd, dyd, k) - 4 -
                             2 * vae2_bn_partial_rows(dyd) * dyd->c;
    float* bp = ws + part_max;
    rc = vae2_bn_stats(dy, dyd, bp, stream);
    if (rc) return rc;
    rc = bias_grad_from_partials(bp, vae2_bn_partial_rows(dyd), dyd->c, dbias, accumulate,
                                 stream);
    if (rc) return rc;
  }
  return 0;
}

int vae2_conv2d_bwd_weight_ld(const float* x, const vae2_act* xd, const float* dy,
                              const vae2_act* dyd, float* dw, int64_t dw_ld, float* dbias,
                              int k, int stride, int pad, int accumulate, float* ws,
                              int64_t ws_size, void* stream) {
  return bwd_weight_impl(x, xd, dy, dyd, dw, dw_ld, dbias, k, stride, pad, accumulate, ws,
                         ws_size, stream, nullptr, 0, "vae2_conv2d_bwd_weight");
}

int vae2_conv2d_bwd_weight_bnin(const float* x, const vae2_act* xd, const float* bn_save,
                                int relu, const float* dy, const vae2_act* dyd, float* dw,
                                float* dbias, int k, int stride, int pad, int accumulate,
                                float* ws, int64_t ws_size, void* stream) {
  const char* fn = "vae2_conv2d_bwd_weight_bnin";
  if (!xd || !bn_save) return fail(fn, "null pointer");
  return bwd_weight_impl(x, xd, dy, dyd, dw, xd->c * k * k, dbias, k, stride, pad, accumulate,
                         ws, ws_size, stream, bn_save, relu, fn);
}

int vae2_conv2d_bwd_weight(const float* x, const vae2_act* xd, const float* dy,
                           const vae2_act* dyd, float* dw, float* dbias, int k,
                           int stride, int pad, int accumulate, float* ws,
                           int64_t ws_size, void* stream) {
  if (!xd) return fail("vae2_conv2d_bwd_weight", "null descriptor");
  return vae2_conv2d_bwd_weight_ld(x, xd, dy, dyd, dw, xd->c * k * k, dbias, k, stride, pad,
                                   accumulate, ws, ws_size, stream);
}
#endif  // VAE2_PART(3)

}  // extern "C"
