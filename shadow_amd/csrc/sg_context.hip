// sg_context.hip -- context lifecycle, error reporting, and the shared
// device-wide exclusive scan used by CSC construction and bucketing.
#include "sg_internal.h"

namespace sg {

// ---- wave64 / block scans ---------------------------------------------------
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// Exclusive block scan over blockDim.x (multiple of 64, <= 1024) values.
// Returns the exclusive prefix; *total receives the block sum.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* total) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t wtot;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t inc = wave_incl_scan(v);
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  if (wid == 0) {
    uint32_t s = lane < nw ? wsum[lane] : 0;
    uint32_t si = wave_incl_scan(s);
    if (lane < nw) wsum[lane] = si - s;
    if (lane == nw - 1) wtot = si;
  }
  __syncthreads();
  uint32_t r = inc - v + wsum[wid];
  *total = wtot;
  __syncthreads();
  return r;
}

constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

__global__ void __launch_bounds__(SCAN_BLOCK) k_scan_reduce(const uint32_t* __restrict__ in, uint32_t n,
                                                            uint32_t* __restrict__ block_sums) {
  size_t base = (size_t)blockIdx.x * SCAN_TILE;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) {
    size_t i = base + (size_t)k * SCAN_BLOCK + threadIdx.x;
    if (i < n) s += in[i];
  }
  uint32_t total;
  (void)block_excl_scan(s, &total);
  if (threadIdx.x == 0) block_sums[blockIdx.x] = total;
}

// Single block: exclusive scan of nb block sums in place; sums[nb] = total.
__global__ void __launch_bounds__(1024) k_scan_blocks(uint32_t* __restrict__ sums, uint32_t nb) {
  uint32_t carry = 0;
  for (uint32_t base = 0; base < nb; base += blockDim.x) {
    uint32_t i = base + threadIdx.x;
    uint32_t v = i < nb ? sums[i] : 0;
    uint32_t total;
    uint32_t ex = block_excl_scan(v, &total);
    if (i < nb) sums[i] = ex + carry;
    carry += total;
  }
  if (threadIdx.x == 0) sums[nb] = carry;
}

__global__ void __launch_bounds__(SCAN_BLOCK) k_scan_down(const uint32_t* __restrict__ in, uint32_t n,
                                                          const uint32_t* __restrict__ block_pref,
                                                          uint32_t* __restrict__ out) {
  // thread t owns SCAN_ITEMS consecutive elements
  size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
  uint32_t v[SCAN_ITEMS];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) {
    size_t i = base + k;
    v[k] = i < n ? in[i] : 0;
    s += v[k];
  }
  uint32_t total;
  uint32_t ex = block_excl_scan(s, &total) + block_pref[blockIdx.x];
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) {
    size_t i = base + k;
    if (i < n) out[i] = ex;
    ex += v[k];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = block_pref[gridDim.x];
}

void exclusive_scan_u32(sg_ctx* ctx, const uint32_t* d_in, uint32_t* d_out, uint32_t n) {
  uint32_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb == 0) {
    SG_HIP(hipMemsetAsync(d_out, 0, sizeof(uint32_t), ctx->stream));
    return;
  }
  uint32_t* sums = ctx->m_scratch.get<uint32_t>((size_t)nb + 1);
  hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(SCAN_BLOCK), 0, ctx->stream, d_in, n, sums);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, ctx->stream, sums, nb);
  hipLaunchKernelGGL(k_scan_down, dim3(nb), dim3(SCAN_BLOCK), 0, ctx->stream, d_in, n, sums, d_out);
  SG_CHECK_LAUNCH();
}

char* stage_acquire(sg_ctx* ctx, int slot, size_t bytes) {
  if (!ctx->stage_used[slot]) SG_HIP(hipEventCreateWithFlags(&ctx->stage_used[slot], hipEventDisableTiming));
  SG_HIP(hipEventSynchronize(ctx->stage_used[slot]));  // the previous copy out of the slot is done
  if (ctx->h_stage_bytes[slot] < bytes) {
    if (ctx->h_stage[slot]) (void)hipHostFree(ctx->h_stage[slot]);
    ctx->h_stage[slot] = nullptr;
    ctx->h_stage_bytes[slot] = 0;
    SG_HIP(hipHostMalloc(&ctx->h_stage[slot], bytes, hipHostMallocDefault));
    ctx->h_stage_bytes[slot] = bytes;
  }
  return (char*)ctx->h_stage[slot];
}

void stage_release(sg_ctx* ctx, int slot) { SG_HIP(hipEventRecord(ctx->stage_used[slot], ctx->stream)); }

void copy_to_host(sg_ctx* ctx, void* dst, const void* src, size_t bytes) {
  SG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
}

static hipEvent_t pool_event(sg_ctx* ctx) {
  if (!ctx->event_pool.empty()) {
    hipEvent_t e = ctx->event_pool.back();
    ctx->event_pool.pop_back();
    return e;
  }
  // timing-only events (read after a stream synchronisation): no system-scope fence at
  // record, whose L2 writeback and invalidation sat inside every timed pair and left the
  // timed kernel a cold L2 (the HIP header recommends this flag for timing events)
  hipEvent_t e;
  SG_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  return e;
}

TimedLaunch::TimedLaunch(sg_ctx* c, const char* name, double work) : ctx(c) {
  if (!ctx->timing) return;
  for (auto& kv : ctx->timers)
    if (kv.first == name) timer = &kv.second;
  if (!timer) {
    ctx->timers.emplace_back(name, KernelTimer());
    timer = &ctx->timers.back().second;
  }
  e0 = pool_event(ctx);
  e1 = pool_event(ctx);
  timer->work += work;
  timer->launches++;
  SG_HIP(hipEventRecord(e0, ctx->stream));
}

void timer_add_work(sg_ctx* ctx, const char* name, double work) {
  if (!ctx->timing) return;
  for (auto& kv : ctx->timers)
    if (kv.first == name) {
      kv.second.work += work;
      return;
    }
  ctx->timers.emplace_back(name, KernelTimer());  // a counter with no launches of its own
  ctx->timers.back().second.work = work;
}

TimedLaunch::~TimedLaunch() {
  if (!timer) return;
  (void)hipEventRecord(e1, ctx->stream);
  timer->pending.emplace_back(e0, e1);
}

// Resolve pending event pairs into total_ms (blocks on the stream).
static void settle_timers(sg_ctx* ctx) {
  SG_HIP(hipStreamSynchronize(ctx->stream));
  for (auto& kv : ctx->timers) {
    for (auto& pr : kv.second.pending) {
      float ms = 0.f;
      SG_HIP(hipEventElapsedTime(&ms, pr.first, pr.second));
      kv.second.total_ms += ms;
      ctx->event_pool.push_back(pr.first);
      ctx->event_pool.push_back(pr.second);
    }
    kv.second.pending.clear();
  }
}

}  // namespace sg

extern "C" {

int32_t sg_abi_version(void) { return SG_ABI_VERSION; }

static thread_local std::string g_create_error;

int32_t sg_ctx_create(int32_t device, sg_ctx** out) {
  if (!out) return SG_ERR_INVALID_ARG;
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || device < 0 || device >= n) {
    g_create_error = std::string("hipGetDeviceCount: ") + hipGetErrorString(e) + ", devices=" +
                     std::to_string(n) + ", requested=" + std::to_string(device);
    return SG_ERR_DEVICE;
  }
  sg_ctx* ctx = new (std::nothrow) sg_ctx();
  if (!ctx) return SG_ERR_OOM;
  ctx->device = device;
  int32_t rc = sg::guarded(ctx, [&] {
    SG_HIP(hipSetDevice(device));
    // a blocking stream: ordered with the legacy default stream, so inputs a
    // caller produced there (torch's default stream) are complete before our
    // kernels read them, and our outputs before its later work reads them
    SG_HIP(hipStreamCreateWithFlags(&ctx->own_stream, hipStreamDefault));
    ctx->stream = ctx->own_stream;
    SG_HIP(hipMalloc(&ctx->round_err, 16));
    SG_HIP(hipMemset(ctx->round_err, 0, 16));
    SG_HIP(hipHostMalloc(&ctx->round_ret, sizeof(sg_round_ret), hipHostMallocMapped | hipHostMallocCoherent));
    SG_HIP(hipHostMalloc(&ctx->apsp_ret, 32, hipHostMallocMapped | hipHostMallocCoherent));
    SG_HIP(hipMalloc(&ctx->sb_ctl, 4 * sg::SB_CTL_STRIDE * 4));
    SG_HIP(hipMemset(ctx->sb_ctl, 0, 4 * sg::SB_CTL_STRIDE * 4));
    int cus = 0;
    SG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    ctx->n_cu = cus;
  });
  if (rc != SG_OK) {
    g_create_error = ctx->last_error;
    delete ctx;
    return rc;
  }
  *out = ctx;
  return SG_OK;
}

void sg_ctx_destroy(sg_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (auto& kv : ctx->timers)
    for (auto& pr : kv.second.pending) {
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
  for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
  if (ctx->round_err) (void)hipFree(ctx->round_err);
  if (ctx->sb_ctl) (void)hipFree(ctx->sb_ctl);
  if (ctx->round_ret) (void)hipHostFree(ctx->round_ret);
  if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
  for (int b = 0; b < 2; b++) {
    if (ctx->stage_done[b]) (void)hipEventDestroy(ctx->stage_done[b]);
    if (ctx->stage_copied[b]) (void)hipEventDestroy(ctx->stage_copied[b]);
  }
  if (ctx->apsp_ret) (void)hipHostFree(ctx->apsp_ret);
  for (auto& b : ctx->net_pool) {
    (void)hipEventDestroy(b.freed);
    (void)hipFree(b.p);
  }
  for (int i = 0; i < 2; i++) {
    if (ctx->stage_used[i]) (void)hipEventDestroy(ctx->stage_used[i]);
    if (ctx->h_stage[i]) (void)hipHostFree(ctx->h_stage[i]);
  }
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  delete ctx;
}

int32_t sg_ctx_set_stream(sg_ctx* ctx, void* hip_stream) {
  if (!ctx) return SG_ERR_INVALID_ARG;
  ctx->stream = hip_stream ? (hipStream_t)hip_stream : ctx->own_stream;
  return SG_OK;
}

void* sg_ctx_stream(const sg_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int32_t sg_ctx_synchronize(sg_ctx* ctx) {
  return sg::guarded(ctx, [&] { SG_HIP(hipStreamSynchronize(ctx->stream)); });
}

const char* sg_ctx_last_error(const sg_ctx* ctx) {
  // NULL: the reason the last sg_ctx_create on this thread failed
  return ctx ? ctx->last_error.c_str() : g_create_error.c_str();
}

void sg_ctx_last_error_pair(const sg_ctx* ctx, uint32_t* row, uint32_t* col) {
  if (row) *row = ctx ? ctx->err_row : 0;
  if (col) *col = ctx ? ctx->err_col : 0;
}

int32_t sg_ctx_enable_timers(sg_ctx* ctx, int32_t enable) {
  return sg::guarded(ctx, [&] {
    sg::settle_timers(ctx);
    ctx->timing = (enable & SG_TIMERS_ON) != 0;
    ctx->count_work = ctx->timing && (enable & SG_TIMERS_COUNT_WORK) != 0;
    for (auto& kv : ctx->timers) kv.second = sg::KernelTimer();
  });
}

int32_t sg_ctx_read_timer(sg_ctx* ctx, const char* kernel, double* total_ms, uint64_t* launches,
                          double* work) {
  return sg::guarded(ctx, [&] {
    sg::settle_timers(ctx);
    double t = 0, w = 0;
    uint64_t n = 0;
    for (auto& kv : ctx->timers)
      if (kernel && kv.first == kernel) {
        t = kv.second.total_ms;
        w = kv.second.work;
        n = kv.second.launches;
      }
    if (total_ms) *total_ms = t;
    if (launches) *launches = n;
    if (work) *work = w;
  });
}

}  // extern "C"
