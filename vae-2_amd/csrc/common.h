// Shared helpers for the gfx950 kernels of libvae2_hip.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <stdio.h>

#include "../../include/vae2_hip.h"

namespace vae2 {

constexpr int kSyncMaxRanks = 8;  // syncbn.hip: ranks of one node

// ------------------------------------------------------------ errors ----
void set_error(const std::string& msg);
int fail(const char* fn, const std::string& msg);  // returns -22
int check_launch(const char* fn);                   // hipGetLastError -> code

// Kernel launch log (vae2_kernel_log): every launch site goes through VAE2_LAUNCH so a
// profiler can attribute the time of each C-ABI call to the kernels it launched.
void note_kernel(const void* host_fn);
#define VAE2_LAUNCH(K, ...)                                         \
  do {                                                              \
    ::vae2::note_kernel(reinterpret_cast<const void*>(K));          \
    hipLaunchKernelGGL(K, __VA_ARGS__);                             \
  } while (0)

#define VAE2_REQUIRE(cond, fn, msg)          \
  do {                                       \
    if (!(cond)) return ::vae2::fail(fn, msg); \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

typedef float f4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------- range-checked loads ----
// A raw buffer load whose byte offset is >= the descriptor's num_records returns 0.
constexpr uint32_t kOOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  uint64_t b = (uint64_t)base;
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  void* pb = (void*)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(pb, (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__device__ __forceinline__ f4 load4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

__device__ __forceinline__ float load1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

// bf16 MFMA operands (v_mfma_f32_16x16x32_bf16): lane (g, r) holds k = 8g .. 8g+7; the
// conv kernels pair two of their fp32 K chunks (4 consecutive k per lane each) into one
// fragment, A and B from the same chunks, so any k order within a chunk pair is shared.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ bf16x8 pack_bf16(f4 a, f4 b) {
  typedef float f8 __attribute__((ext_vector_type(8)));
  const f8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_convertvector(v, bf16x8);  // v_cvt_pk_bf16_f32 (RNE, NaN kept)
}

__device__ __forceinline__ void store1(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, 0);
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void store4(__amdgpu_buffer_rsrc_t r, uint32_t off, f4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 0);
}

__device__ __forceinline__ uint32_t load_u8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
}

__device__ __forceinline__ d2 load_d2(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// The first n (1..4) channels of a channel quad at byte offset off, without branches: a
// whole quad as one 16-byte store, a partial one as (2 +) 1 stores; the unused forms get an
// out-of-range offset (dropped).  Channels past n are never written (they may belong to
// the next tensor of a concatenation buffer).
__device__ __forceinline__ void store_quad(__amdgpu_buffer_rsrc_t r, uint32_t off, f4 v, int n) {
  store4(r, n >= 4 ? off : kOOB, v);
  // (the pair as a shuffle of the bit-cast quad: an element-wise {v[0], v[1]} initializer
  //  was compiled to {v[0], v[0]} by hipcc 7.2 here -- channel 1 of every partial quad lost)
  const u32x4 w = __builtin_bit_cast(u32x4, v);
  const u32x2 lo = __builtin_shufflevector(w, w, 0, 1);
  __builtin_amdgcn_raw_buffer_store_b64(lo, r, (n & 2) && n < 4 ? off : kOOB, 0, 0);
  store1(r, (n & 1) ? off + 4u * (uint32_t)(n & 2) : kOOB, (n & 2) ? v[2] : v[0]);
}

// Bijective blockIdx remap (T1): blocks are dealt round-robin over the 8 XCDs, so
// logical tiles are re-numbered to make each XCD own a contiguous run of tiles
// (vertically adjacent image rows share that XCD's L2).  Speed only.
__device__ __forceinline__ int xcd_remap(int orig, int n) {
  const int q = n >> 3, rr = n & 7, x = orig & 7;
  return (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (orig >> 3);
}

// 4 x 4 transpose across the 4 lanes of a lane quad (DPP quad_perm, no LDS): lane k's
// v[e] becomes lane e's former v[k].  A 16x16 MFMA accumulator (lane (g, r) = column r,
// rows 4g..4g+3) then has lane (g, 4Q + k) holding row 4g + k, columns 4Q..4Q+3.
__device__ __forceinline__ float dpp_xor1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v),
                                                            0xB1, 0xF, 0xF, true));
}
__device__ __forceinline__ float dpp_xor2(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v),
                                                            0x4E, 0xF, 0xF, true));
}
__device__ __forceinline__ void quad_transpose(f4& v, int k) {
  const bool o = k & 1;
  float a = dpp_xor1(o ? v[0] : v[1]), b = dpp_xor1(o ? v[2] : v[3]);
  if (o) { v[0] = a; v[2] = b; } else { v[1] = a; v[3] = b; }
  const bool h = k & 2;
  a = dpp_xor2(h ? v[0] : v[2]);
  b = dpp_xor2(h ? v[1] : v[3]);
  if (h) { v[0] = a; v[1] = b; } else { v[2] = a; v[3] = b; }
}

// ------------------------------------------------------- activations ----
// Device-side copy of vae2_act with 32-bit-safe strides kept in 64-bit.
struct Act {
  int64_t n, h, w, c, ps;
};

inline Act to_act(const vae2_act* d) { return Act{d->n, d->h, d->w, d->c, d->ps}; }

inline bool act_ok(const vae2_act* d) {
  return d && d->n > 0 && d->h > 0 && d->w > 0 && d->c > 0 && d->ps >= d->c;
}

inline int64_t act_pixels(const vae2_act* d) { return d->n * d->h * d->w; }
inline int64_t act_elems(const vae2_act* d) { return d->n * d->h * d->w * d->c; }

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Division by a runtime constant via multiply-high (valid for n < 2^31).
struct FastDiv {
  uint32_t d, m, s;
  FastDiv() : d(1), m(0), s(0) {}
  explicit FastDiv(uint32_t div) : d(div) {
    for (s = 0; s < 32; ++s)
      if ((1u << s) >= d) break;
    uint64_t one = 1;
    m = (uint32_t)(((one << 32) * ((one << s) - d)) / d + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    return (__umulhi(n, m) + n) >> s;
  }
};

// ------------------------------------------------- bilinear helpers ----
// PyTorch's area_pixel_compute_source_index for align_corners=False, in fp32.
struct Lerp {
  int i0, i1;
  float l0, l1;
};

__device__ __forceinline__ Lerp lerp_index(int dst, int in_size, float scale) {
  float src = scale * ((float)dst + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  int i0 = (int)src;
  if (i0 > in_size - 1) i0 = in_size - 1;
  int ip = (i0 < in_size - 1) ? 1 : 0;
  Lerp l;
  l.i0 = i0;
  l.i1 = i0 + ip;
  l.l1 = src - (float)i0;
  l.l0 = 1.f - l.l1;
  return l;
}

// Weight with which output coordinate `o` reads input coordinate `i`.
__device__ __forceinline__ float lerp_weight(int o, int in_size, float scale, int i) {
  Lerp l = lerp_index(o, in_size, scale);
  float w = 0.f;
  if (l.i0 == i) w += l.l0;
  if (l.i1 == i) w += l.l1;
  return w;
}

// Exact 2^k ratios (the HRNet branches of a power-of-two image): source column i of
// a bilinear upsample by F receives the 2F output pixels F*i + d, d = -F/2 .. 3F/2-1,
// with the hat weight 1 - |2d + 1 - F| / 2F (interpolate's lerp weights, exact in
// fp32); at the image edges the forward's clamped tap lands on column 0 / w-1, i.e.
// the virtual columns -1 and w are folded into them.  Same rule vertically.
__device__ constexpr float hat_w(int d, int f) {
  return 1.f - (float)(2 * d + 1 - f < 0 ? f - 1 - 2 * d : 2 * d + 1 - f) / (float)(2 * f);
}

// Internal (heads.hip): the fuse layers' pow2 upsampling adjoint through the one-pass
// kernel, or -1 when its shape rules do not hold.
int adj3_fuse_launch(const float* dy, const vae2_act* dyd, int n, float* const* dxs,
                     const vae2_act* dxds, const float* betas, hipStream_t st);
extern int g_relu_dual_q;  // heads.hip: vae2_heads_set_algo bit 7 clears it

// Internal (wgrad_narrow.hip): the narrow-channel 3x3 weight gradient.  _splits: partial
// slabs it writes for this layer (0: not handled); _launch: writes them into part
// ([splits][cout][9 * cin4]) and returns their number, 0 when not handled, < 0 on error.
int64_t wgrad3n_splits(const vae2_act* xd, const vae2_act* dyd);
int wgrad3n_launch(const float* x, const vae2_act* xd, const float* dy, const vae2_act* dyd,
                   float* part, const float* isave, int irelu, uint32_t x_bytes,
                   uint32_t dy_bytes, hipStream_t s);

// Internal (dconv_stream.hip): the streaming direct 3x3 kernel of the 18 / 36-channel
// branches.  _shape: it takes this (input, output) pair; _rows: its BatchNorm partial rows
// (workgroups); _launch: 1 when launched, 0 when the shape is not its own.
extern int g_dconv_stream, g_dconv_stream_wpc, g_dconv_stream_bl, g_dconv_stream_spb,
    g_wgrad_narrow_tps, g_bn_blocks, g_bn_apply_res, g_fuse_quad;
bool dconv3s_shape(const vae2_act* ad, const vae2_act* yd);
int64_t dconv3s_rows(const vae2_act* ad, const vae2_act* yd);
int dconv3s_launch(const float* a, const vae2_act* ad, const float* wp, uint32_t w_bytes,
                   const float* bias, float* y, const vae2_act* yd, float beta, float* stats,
                   bool flip, const float* isave, int irelu, const float* bx, int bx_ps,
                   int brelu, const float* bsave, uint32_t bx_bytes, uint32_t a_bytes,
                   hipStream_t s);

// Internal (not part of the public ABI): dbias (+)= column sums from BN-style partials.
int bias_grad_from_partials(const float* partials, int64_t rows, int64_t c,
                            float* dbias, int accumulate, void* stream);

// Grid size for element-wise kernels: one element (or quad) per thread up to 16.7 M of
// them, then grid-striding.  (A thread that loops stores, then issues its next loads:
// vmcnt counts stores too, so every iteration after the first also waits for the previous
// iteration's store -- the 8192-block cap made the 128x256 fuse sums loop 2-3 times.)
inline unsigned ew_blocks(int64_t n, int threads = 256, int64_t cap = 65536) {
  int64_t b = ceil_div(n, threads);
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (unsigned)b;
}

}  // namespace vae2
