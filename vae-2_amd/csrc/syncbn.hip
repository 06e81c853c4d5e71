// One-shot peer all-reduce of the SyncBatchNorm statistics between the ranks of one node.
//
// The reference converts every BatchNorm to SyncBatchNorm (tools/train.py:216-218), whose
// forward and backward each all-reduce a few KB per layer; vae2/dist.py batches them into
// one exchange per BN depth level (448 + 18 per step).  Through RCCL each is a ring all-reduce
// of a tiny buffer: latency-bound, ~10-25 us on 8 GPUs.  Here each exchange is ONE kernel:
//
//   1. every rank stores its payload into slot (seq & 1) of EVERY rank's receive area
//      (IPC-mapped device memory, the peers over xGMI; system-scope stores),
//   2. releases it (system-scope fence) and raises its arrival flag in every area,
//   3. waits until all `world` flags of its own area reach seq,
//   4. sums the world payloads in rank order -- the same doubles on every rank.
//
// Two slots suffice: a rank reuses slot s only for exchange seq + 2, after it saw every
// peer's flag for seq + 1, which each peer raised after finishing its reads of exchange seq
// (stream order).  seq lives in device memory (incremented by the kernel), so a captured
// HIP graph replays correctly.  Every wait is bounded (s_memrealtime, 60 s): a missing peer
// sets the area's error word and the kernel exits instead of hanging the GPU.
//
// Failures are sticky and visible in the data: a timed-out exchange writes NaN into the
// caller's buffer (the statistics become NaN, so the step's NaN/Inf checks see it even
// where nobody reads the error word), and every later exchange on this comm finds the
// error word set at entry, copies nothing, raises no flag and writes NaN again -- a rank
// never goes on pairing its payloads with the wrong exchange of its peers.  The receive
// areas are uncached device memory (hipDeviceMallocUncached), so the peers' system-scope
// stores over xGMI and this rank's polling loads meet in HBM, not in a stale L2 line.
//
// A flag word is seq | n << 40: a rank whose peer arrived at the same sequence number with
// a different payload length (the ranks' exchange sequences diverged -- e.g. one rank's
// control flow skipped a layer) fails that exchange instead of summing unrelated payloads.
//
// Area layout (bytes): [0, 64) control {seq, error}; [64, 64 + 16 * world) flags[2][world]
// (u64); from kRecvOff: recv[2][world][max_elems] doubles.
#include <hip/hip_runtime.h>

#include <string.h>

#include "common.h"

struct vae2_syncbn_comm {
  int rank, world;
  int64_t max_elems;
  uint64_t timeout_ticks;              // s_memrealtime ticks (100 MHz) before giving up
  void* area;                          // own area (allocated here, freed by destroy)
  void* peers[vae2::kSyncMaxRanks];    // every rank's area mapped in this process
  bool opened[vae2::kSyncMaxRanks];    // peers[r] from hipIpcOpenMemHandle
};

namespace vae2 {

namespace {

constexpr int64_t kRecvOff = 4096;
// s_memrealtime at 100 MHz: 60 s (ranks legitimately drift apart by seconds at start-up:
// module loading, graph capture; a timed-out exchange corrupts the sequence, so the host
// checks the error word -- vae2.dist.syncbn_check -- and fails loudly)
constexpr uint64_t kTimeoutTicks = 6000000000ull;
constexpr double kTicksPerSecond = 1.0e8;
constexpr uint64_t kSeqMask = (1ull << 40) - 1;

struct SyncArgs {
  char* peers[kSyncMaxRanks];
  int rank, world;
  int64_t max_elems;
  uint64_t timeout_ticks;
  double* buf;
  int n;
};

__device__ __forceinline__ uint64_t* ctrl(char* a) { return reinterpret_cast<uint64_t*>(a); }
__device__ __forceinline__ uint64_t* flags(char* a) { return reinterpret_cast<uint64_t*>(a + 64); }
__device__ __forceinline__ double* recv(char* a) { return reinterpret_cast<double*>(a + kRecvOff); }

__global__ __launch_bounds__(256) void syncbn_allreduce_kernel(SyncArgs p) {
  __shared__ uint64_t sseq;
  __shared__ int sfail;
  char* own = p.peers[p.rank];
  if (threadIdx.x == 0) {
    // sticky failure: an earlier exchange of this comm timed out -> no payload, no flag
    const uint64_t err = __hip_atomic_load(ctrl(own) + 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    sfail = err != 0;
    if (!sfail) {
      const uint64_t s = ctrl(own)[0] + 1;  // only this (stream-ordered) kernel writes it
      ctrl(own)[0] = s;
      sseq = s;
    }
  }
  __syncthreads();
  if (sfail) {
    for (int i = threadIdx.x; i < p.n; i += blockDim.x) p.buf[i] = __builtin_nan("");
    return;
  }
  const uint64_t seq = sseq;
  const int slot = (int)(seq & 1);
  // 1. the payload into every rank's slot (system scope: visible to the peer's loads)
  for (int r = 0; r < p.world; ++r) {
    double* dst = recv(p.peers[r]) + ((int64_t)slot * p.world + p.rank) * p.max_elems;
    for (int i = threadIdx.x; i < p.n; i += blockDim.x)
      __hip_atomic_store(dst + i, p.buf[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: this thread's stores are
  __syncthreads();                                // complete before the flags below
  // 2. arrival flags (thread r raises ours in rank r's area)
  if ((int)threadIdx.x < p.world) {
    __hip_atomic_store(flags(p.peers[threadIdx.x]) + slot * p.world + p.rank,
                       seq | ((uint64_t)p.n << 40), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for every rank's flag in our area (bounded), then check its payload length
  if ((int)threadIdx.x < p.world) {
    uint64_t* f = flags(own) + slot * p.world + threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t v;
    bool late = false;
    while (((v = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) & kSeqMask) <
           seq) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > p.timeout_ticks) {
        late = true;
        break;
      }
    }
    if (late || (v >> 40) != (uint64_t)p.n) sfail = 1;
  }
  __syncthreads();
  if (sfail) {  // the statistics of this exchange are undefined: make them NaN
    if (threadIdx.x == 0)
      __hip_atomic_fetch_or(ctrl(own) + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int i = threadIdx.x; i < p.n; i += blockDim.x) p.buf[i] = __builtin_nan("");
    return;
  }
  // 4. the world payloads in rank order (system-scope loads: the peers wrote them)
  const double* src = recv(own) + (int64_t)slot * p.world * p.max_elems;
  for (int i = threadIdx.x; i < p.n; i += blockDim.x) {
    double s = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (int r = 1; r < p.world; ++r)
      s += __hip_atomic_load(src + (int64_t)r * p.max_elems + i, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    p.buf[i] = s;
  }
}

int64_t area_bytes(int world, int64_t max_elems) {
  return kRecvOff + 2 * (int64_t)world * max_elems * (int64_t)sizeof(double);
}

}  // namespace
}  // namespace vae2

using namespace vae2;

extern "C" {

int64_t vae2_syncbn_comm_bytes(int world, int64_t max_elems) {
  if (world < 1 || world > kSyncMaxRanks || max_elems < 1) return 0;
  return area_bytes(world, max_elems);
}

int vae2_syncbn_comm_init(int rank, int world, int64_t max_elems, void* handle_out,
                          vae2_syncbn_comm** out) {
  const char* fn = "vae2_syncbn_comm_init";
  VAE2_REQUIRE(out && handle_out && world >= 1 && world <= kSyncMaxRanks && rank >= 0 &&
                   rank < world && max_elems >= 1 && max_elems <= (1 << 24),
               fn, "bad arguments (world <= 8, 0 <= rank < world, 1 <= max_elems <= 2^24)");
  *out = nullptr;
  vae2_syncbn_comm* c = new vae2_syncbn_comm();
  c->rank = rank;
  c->world = world;
  c->max_elems = max_elems;
  c->timeout_ticks = kTimeoutTicks;
  const int64_t bytes = area_bytes(world, max_elems);
  // uncached: the peers' xGMI stores and this rank's polling loads meet in HBM
  hipError_t e = hipExtMallocWithFlags(&c->area, (size_t)bytes, hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(c->area, 0, (size_t)bytes);
  hipIpcMemHandle_t h;
  if (e == hipSuccess) e = hipIpcGetMemHandle(&h, c->area);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    if (c->area) (void)hipFree(c->area);
    delete c;
    return fail(fn, hipGetErrorString(e));
  }
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle size");
  memset(handle_out, 0, 64);
  memcpy(handle_out, &h, sizeof(h));
  c->peers[rank] = c->area;
  *out = c;
  return 0;
}

int vae2_syncbn_comm_connect(vae2_syncbn_comm* c, const void* handles) {
  const char* fn = "vae2_syncbn_comm_connect";
  VAE2_REQUIRE(c && handles, fn, "null argument");
  for (int r = 0; r < c->world; ++r) {
    if (r == c->rank || c->peers[r]) continue;
    hipIpcMemHandle_t h;
    memcpy(&h, static_cast<const char*>(handles) + 64 * r, sizeof(h));
    void* p = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return fail(fn, std::string("rank ") + std::to_string(r) + ": " +
                                             hipGetErrorString(e));
    c->peers[r] = p;
    c->opened[r] = true;
  }
  return 0;
}

int vae2_syncbn_allreduce(vae2_syncbn_comm* c, double* buf, int64_t n, void* stream) {
  const char* fn = "vae2_syncbn_allreduce";
  VAE2_REQUIRE(c && buf && n >= 0 && n <= c->max_elems, fn, "bad arguments (n <= max_elems)");
  SyncArgs a{};
  for (int r = 0; r < c->world; ++r) {
    VAE2_REQUIRE(c->peers[r], fn, "not connected (vae2_syncbn_comm_connect)");
    a.peers[r] = static_cast<char*>(c->peers[r]);
  }
  a.rank = c->rank;
  a.world = c->world;
  a.max_elems = c->max_elems;
  a.timeout_ticks = c->timeout_ticks;
  a.buf = buf;
  a.n = (int)n;
  VAE2_LAUNCH(syncbn_allreduce_kernel, dim3(1), dim3(256), 0, as_stream(stream), a);
  return check_launch(fn);
}

int vae2_syncbn_comm_set_timeout(vae2_syncbn_comm* c, double seconds) {
  const char* fn = "vae2_syncbn_comm_set_timeout";
  VAE2_REQUIRE(c && seconds > 0.0 && seconds <= 3600.0, fn, "bad arguments (0 < seconds <= 3600)");
  c->timeout_ticks = (uint64_t)(seconds * kTicksPerSecond);
  return 0;
}

int vae2_syncbn_comm_error(vae2_syncbn_comm* c, int64_t* host_out) {
  const char* fn = "vae2_syncbn_comm_error";
  VAE2_REQUIRE(c && host_out, fn, "null argument");
  uint64_t v = 0;
  const hipError_t e = hipMemcpy(&v, static_cast<char*>(c->area) + 8, 8, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return fail(fn, hipGetErrorString(e));
  *host_out = (int64_t)v;
  return 0;
}

int vae2_syncbn_comm_destroy(vae2_syncbn_comm* c) {
  if (!c) return 0;
  for (int r = 0; r < c->world; ++r)
    if (c->opened[r]) (void)hipIpcCloseMemHandle(c->peers[r]);
  if (c->area) (void)hipFree(c->area);
  delete c;
  return 0;
}

}  // extern "C"
