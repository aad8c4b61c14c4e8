// sg_internal.h -- host-side runtime shared by the HIP translation units:
// context, grow-only device workspace, error plumbing.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <new>
#include <stdexcept>
#include <string>
#include <atomic>
#include <deque>
#include <memory>
#include <vector>

#include "../../include/shadow_gpu.h"

namespace sg {

// Status-carrying exception; converted to a status code at the C boundary.
struct Error : std::runtime_error {
  int32_t code;
  uint32_t row, col;
  Error(int32_t c, const std::string& m, uint32_t r = 0, uint32_t k = 0)
      : std::runtime_error(m), code(c), row(r), col(k) {}
};

#define SG_HIP(expr)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) {                                                                 \
      if (e_ == hipErrorOutOfMemory) throw ::sg::Error(SG_ERR_OOM, std::string(#expr) + ": out of device memory"); \
      throw ::sg::Error(SG_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    }                                                                                       \
  } while (0)

#define SG_CHECK_LAUNCH() SG_HIP(hipGetLastError())

// Grow-only device buffer.  Growth is the only path that allocates, so a
// steady-state round never calls hipMalloc.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* get(size_t count) {
    size_t bytes = count * sizeof(T);
    if (bytes == 0) bytes = 16;
    if (bytes > cap) {
      release();
      SG_HIP(hipMalloc(&p, bytes));
      cap = bytes;
    }
    return static_cast<T*>(p);
  }
};

// Per-kernel timer: HIP events recorded on the context stream around each
// launch of an instrumented kernel (bench.py reads the average launch time and
// the algorithmic work the launch site declares).
struct KernelTimer {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  double total_ms = 0.0;
  double work = 0.0;  // algorithmic units (relaxations / bytes), summed over launches
  uint64_t launches = 0;
};


}  // namespace sg

struct sg_round_ret {
  unsigned long long stats[3];  // n_delivered, min deliver time, min used latency
  uint32_t err;
  uint32_t overflow;  // a bucketing region overflowed: the scan path must run
  // sg_deliver_bucket_padded: this rank's receive count from each rank, and the
  // largest count any rank sent any rank (over the padded capacity: exchange again)
  uint32_t recv_cnt[64];
  uint32_t pair_max;
  uint32_t pad_;
};

struct sg_ctx {
  int device = 0;
  unsigned long long* pair_count = nullptr;  // sg_ctx_set_packet_counters: per table cell (device), or null
  uint64_t pair_count_cells = 0;
  uint64_t net_serial = 0;   // the last sg_net serial handed out
  uint64_t dense_owner = 0;  // the net whose arcs r_dense holds sorted (0: none)
  uint32_t dense_gen = 0;    // stamp of the dense search's seed-row marks in r_dense (0: none valid)
  uint64_t band_owner = 0;   // the net whose degree-class numbering r_band holds (0: none)
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  int n_cu = 256;
  std::string last_error;
  uint32_t err_row = 0, err_col = 0;
  // routing workspace
  sg::DevBuf r_dist, r_dist2, r_flags, r_used, r_err, r_self, r_pair_cnt, r_pair_edge, r_map, r_out_lat,
      r_out_loss, r_misc, r_dirty, r_work, r_items, r_plan, r_dense, r_done, r_bucket, r_band;
  // delivery workspace
  sg::DevBuf d_seg, d_dst, d_cnt, d_cur, d_keys, d_vals, d_keys2, d_vals2, d_keys3, d_keys4, d_misc,
      d_scan, d_lists, d_lists2, d_ctr0, d_blk, d_spill;
  sg::DevBuf m_scratch;
  // sg_routing_info_fill: double-buffered device row blocks, copied to the host
  // on copy_stream while the next block computes
  sg::DevBuf r_stage_lat[2], r_stage_loss[2], r_stage_pack[2];
  hipStream_t copy_stream = nullptr;
  bool in_fill = false;  // inside sg_routing_info_fill (selects the row-block kernel symbols)
  hipEvent_t stage_done[2] = {nullptr, nullptr}, stage_copied[2] = {nullptr, nullptr};
  // Round control: round_err (device, zeroed at creation) collects the source
  // phase's error flags; the stats kernel hands them to the host and clears
  // them for the next round.  round_ret (pinned, mapped host memory) receives
  // the round's stats and error flags straight from that kernel: no copies.
  uint32_t* round_err = nullptr;
  sg_round_ret* round_ret = nullptr;
  // Region bucketing counters, two parities of [SB_SUB x SB_MAX counts + overflow
  // flag] (zeroed at creation; each call's sort kernel clears the other parity),
  // then two parities for the coarse level of two-level scatters (cleared by the
  // second level's kernel).
  uint32_t* sb_ctl = nullptr;
  uint32_t sb_parity = 0, sb_parity_c = 0;
  sg::DevBuf d_cd, d_ct, d_ck, d_ci;  // coarse-level runs of a two-level scatter
  // APSP (pinned host-mapped, 32 B): [0] the slab's active-batch count of the next
  // pass (k_active_list, each pass-chunk end); [4] the LDS search's flagged rows and
  // [2..3] the self-loop check's first failure (k_build_finish, the build's end)
  uint32_t* apsp_ret = nullptr;
  // sg_routing_build's self-loop check (graph/mod.rs:210-217), folded into the LDS
  // search's final kernel when it runs: the inputs, and the result once read
  const uint32_t* self_used = nullptr;
  uint32_t self_n = 0;
  const uint32_t* self_cnt = nullptr;
  bool self_done = false;
  unsigned long long self_first = ~0ull;
  // sg_net device blocks released by sg_net_destroy, reused by the next sg_net_create
  // (a simulation that builds one graph and one table pays no hipMalloc / hipFree,
  // whose implicit device synchronisation cost ~0.2 ms each); `freed` orders the
  // reuse after the last work queued on the released block
  struct NetBlock {
    void* p;
    size_t bytes;
    hipEvent_t freed;
  };
  std::vector<NetBlock> net_pool;
  // pinned staging of a new graph's edge arrays (one H2D copy); `stage_used` marks
  // when the last copy out of it completed
  // (slot 0: edges; slot 1: a build's used-node list)
  void* h_stage[2] = {nullptr, nullptr};
  size_t h_stage_bytes[2] = {0, 0};
  hipEvent_t stage_used[2] = {nullptr, nullptr};
  // kernel timers (off unless sg_ctx_enable_timers)
  bool timing = false;
  bool count_work = false;  // SG_TIMERS_COUNT_WORK
  std::deque<std::pair<std::string, sg::KernelTimer>> timers;  // deque: stable addresses
  std::vector<hipEvent_t> event_pool;
};

// Device-resident network graph (sg_routing.hip builds it).
struct sg_net {
  sg_ctx* ctx = nullptr;
  uint64_t serial = 0;  // unique per context: who owns the context's sorted-arc workspace (sg_dense.hip)
  uint32_t n_nodes = 0, n_edges = 0, n_arcs = 0;
  bool directed = false;
  // the arcs' smallest latency and mean latency (each clamped to LAT32_SAT), taken on the host
  // for graphs the bucketed search takes (sg_bucket.hip sizes its bucket width from them)
  uint32_t arc_lat_min = 0;
  double arc_lat_mean = 0.0;
  std::vector<uint32_t> gml_id;
  // GML edge list (device)
  uint32_t* e_src = nullptr;
  uint32_t* e_dst = nullptr;
  uint64_t* e_lat = nullptr;
  float* e_loss = nullptr;
  // in-arc CSC without self-loops (device)
  uint32_t* in_off = nullptr;  // n_nodes + 1
  uint32_t* in_src = nullptr;
  uint64_t* in_lat = nullptr;    // exact latency (wide kernel)
  float* in_om = nullptr;        // 1f32 - loss
  uint4* in_rec = nullptr;       // per in-arc (source, destination, latency32, bits(1f32 - loss))
  bool csc = false;              // the in-arc arrays above are built (ensure_csc, on first use)
  // out-arc CSR without self-loops (device), for the per-source LDS search
  // (sg_sssp.hip): out_arc = 3 u32 per arc (head node, latency32, bits(1f32 - loss))
  uint32_t* out_off = nullptr;  // n_nodes + 1
  uint32_t* out_arc = nullptr;
  // self-loops
  uint32_t* self_cnt = nullptr;
  uint32_t* self_edge = nullptr;
  void* mem = nullptr;  // one device block holding every array above (from the context's pool)
  size_t mem_bytes = 0;
  ~sg_net() {
    if (mem) (void)hipFree(mem);  // (sg_net_destroy hands it back to the pool instead)
  }
};

// Host-resident dense RoutingInfo (sg_route_info.hip).
struct sg_routing_info {
  uint32_t n = 0;
  std::vector<uint32_t> node_ids;
  // n x n cells (latency << 32) | bits(loss), pinned when a device was present at
  // creation; a cell whose latency half is SG_CELL_WIDE has its u64 latency in
  // `wide` (sorted by cell index)
  uint64_t* cell = nullptr;
  bool pinned = false;
  struct Wide {
    uint64_t cell;
    uint64_t lat;
  };
  std::vector<Wide> wide;
  // per row: 0 not written, 1 written with its smallest latency in row_min, 2 written by a
  // fill (row_min not kept; computed once if set_rows later needs it); all written -> filled
  std::vector<uint8_t> row_set;
  std::vector<uint64_t> row_min;
  uint32_t rows_set = 0;
  bool filled = false;
  uint64_t min_lat = UINT64_MAX;
  // GML id -> row: dense window [id_base, id_base + id_span) or sorted (id, row) pairs
  uint32_t id_base = 0, id_span = 0;
  std::vector<uint32_t> id_dense;
  std::vector<std::pair<uint32_t, uint32_t>> id_sorted;
  // address (host byte order) -> row (IpAssignment::get_node, then the id map)
  uint32_t ip_base = 0, ip_span = 0;
  std::vector<uint32_t> ip_dense;
  std::vector<std::pair<uint32_t, uint32_t>> ip_sorted;
  // increment_packet_count: n x n saturating counters, allocated on first use
  std::atomic<uint64_t*> counters{nullptr};
  ~sg_routing_info();
};

namespace sg {

// Run `fn` with the context's device current; map exceptions to status codes.
template <class F>
int32_t guarded(sg_ctx* ctx, F&& fn) {
  if (!ctx) return SG_ERR_INVALID_ARG;
  try {
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != ctx->device) SG_HIP(hipSetDevice(ctx->device));
    fn();
    ctx->last_error.clear();
    ctx->err_row = ctx->err_col = 0;
    return SG_OK;
  } catch (const Error& e) {
    ctx->last_error = e.what();
    ctx->err_row = e.row;
    ctx->err_col = e.col;
    return e.code;
  } catch (const std::bad_alloc&) {
    ctx->last_error = "host out of memory";
    return SG_ERR_OOM;
  } catch (const std::exception& e) {
    ctx->last_error = e.what();
    return SG_ERR_DEVICE;
  }
}

// Region bucketing counters per parity: 8 sub-counters (one per XCD) x SB_MAX
// (4096) super-buckets + an overflow flag.
constexpr uint32_t SB_SUB = 8;
constexpr uint32_t SB_CTL_STRIDE = SB_SUB * 4096 + 1;

inline unsigned grid_for(size_t n, unsigned block, unsigned cap = 1u << 20) {
  size_t g = (n + block - 1) / block;
  if (g == 0) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// Exclusive scan of n u32 values (device, in -> out, out has n+1 entries, out[n] = total).
void exclusive_scan_u32(sg_ctx* ctx, const uint32_t* d_in, uint32_t* d_out, uint32_t n);

// Group offsets of a key array grouped by ascending key (sg_deliver.hip's
// k_host_off): off[g] = first index whose key >= g, g = 0..n_groups.  err bit
// 1: not grouped ascending; bit 2: a key >= n_groups.
void launch_group_offsets(sg_ctx* ctx, const uint32_t* key, uint32_t n, uint32_t n_groups, uint32_t* off,
                          uint32_t* err);

// Read a few scalars back (blocking on the context stream).
void copy_to_host(sg_ctx* ctx, void* dst, const void* src, size_t bytes);

// Pinned staging for host-to-device copies (a pageable source costs the runtime's own
// staging and ~20 us): stage_acquire waits until the slot's previous copy has left it
// and returns it (grown to `bytes`); stage_release after the hipMemcpyAsync out of it.
char* stage_acquire(sg_ctx* ctx, int slot, size_t bytes);
void stage_release(sg_ctx* ctx, int slot);

// Add algorithmic work to a timer after the fact (e.g. a device-side count).
void timer_add_work(sg_ctx* ctx, const char* name, double work);

// RAII bracket for one instrumented launch: `TimedLaunch t(ctx, "k_walk", work);`
// before the launch; the end event is recorded when `t` goes out of scope.
struct TimedLaunch {
  sg_ctx* ctx;
  KernelTimer* timer = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  TimedLaunch(sg_ctx* c, const char* name, double work);
  ~TimedLaunch();
};

// Per-source LDS-resident shortest paths (sg_sssp.hip).  Rows [row_begin,
// row_end) of the table, one workgroup each; or, with blk_rows, the n_blk rows
// listed there (absolute, within [row_begin, row_end)).  ub_row / ub_w (per
// workgroup, SSSP_KB_MAX each, optional): rows of out-neighbours s' already in
// the table (~0u: none) and the arc latencies s -> s'; the search starts every
// key at min over them of (w + D[s'][v]) + 1 instead of infinity.  A bound row
// whose ub_row entry carries SSSP_UB_EXACT (a zero-loss arc s -> s', every node a
// used node) also seeds exact keys (w + D[s'][v].lat, D[s'][v].loss); see
// sg_sssp.hip "Exact seeds".  The bound rows must be final before the launch
// (an earlier launch on the stream).
// Per-source search of dense graphs, settling by rounds and relaxing only the arcs
// below the round's largest unsettled latency (sg_dense.hip): rows [row_begin,
// row_end); sat_row (zeroed by the caller) receives 1 for rows needing the wide
// kernel.  Sorts every node's out-arcs by latency on the stream first.  work
// (optional, WORK_SHARDS counters): arcs relaxed.
constexpr uint32_t DENSE_MAX = 4096;
bool sssp_dense_fits(uint32_t n_nodes);
void launch_sssp_dense(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used, uint32_t row_begin,
                       uint32_t row_end, uint64_t* out_lat, float* out_loss, uint32_t* sat_row,
                       unsigned long long* work);

// Per-source delta-stepping search of sparse graphs past the LDS search (sg_bucket.hip): rows
// [row_begin, row_end); sat_row (zeroed by the caller) receives 1 for rows needing the wide
// kernel, 2 for rows whose search gave up.  work / diag optional (relaxations; [buckets,
// entries, far steps, pops]).
bool sssp_bucket_fits(uint32_t n_nodes);
void launch_sssp_bucket(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used, uint32_t row_begin,
                        uint32_t row_end, uint64_t* out_lat, float* out_loss, uint32_t* sat_row,
                        unsigned long long* work, unsigned long long* diag);

constexpr int SSSP_KB_MAX = 8;
constexpr uint32_t SSSP_UB_EXACT = 0x80000000u;  // bound rows per bounded search (sg_sssp.hip SSSP_KB)
bool sssp_lds_fits(uint32_t n_nodes);
// build the in-arc CSC of a net on its first use (sg_routing.hip; the upload writes the out-arcs only)
void ensure_csc(sg_ctx* ctx, sg_net* net);

void launch_sssp_lds(sg_ctx* ctx, const uint32_t* out_off, const uint32_t* out_arc, uint32_t n, uint32_t n_arcs,
                     const uint32_t* d_used, uint32_t n_used, uint32_t row_begin, uint32_t row_end,
                     const uint32_t* self_edge, const uint64_t* e_lat, const float* e_loss, uint64_t* out_lat,
                     float* out_loss, uint32_t* sat_row, uint32_t delta, unsigned long long* work,
                     unsigned long long* diag, const uint32_t* blk_rows = nullptr, uint32_t n_blk = 0,
                     const uint32_t* ub_row = nullptr, const uint32_t* ub_w = nullptr,
                     const uint32_t* plan_ctl = nullptr, int plan_ph = 0, uint32_t* plan_ctr = nullptr,
                     uint32_t* done = nullptr);

// The LDS search's phase plan, built on the device (sg_plan.hip) on the context
// stream: phase p's rows are list[ctl[2p] .. + ctl[2p + 1]) (absolute row indices),
// their SSSP_KB_MAX bound rows and latencies at the same list positions of ub_row /
// ub_w; ctr[2p .. 2p + 2) are the phase launch's claim counters (zeroed).
struct SsspDevPlan {
  int n_phase = 0;
  uint32_t* list = nullptr;
  uint32_t* ub_row = nullptr;
  uint32_t* ub_w = nullptr;
  uint32_t* ctl = nullptr;
  uint32_t* ctr = nullptr;
  bool landmarks = false;  // phase 0 = landmark rows; phase 1's bounds come from them (sssp_landmark_bounds)
  unsigned rows_grid = 0;  // sssp_landmark_bounds' grid (one thread per row of the block)
};
constexpr int SSSP_PHASES_MAX = 6;
SsspDevPlan sssp_device_plan(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used, uint32_t row_begin,
                             uint32_t row_end, int n_phase, int kb, bool exact, int hops, uint32_t n_land,
                             uint32_t* zero_rows = nullptr, uint32_t* zero_rows2 = nullptr);
// After phase 0 (the landmarks) ran: phase 1's bound rows from the landmark rows' columns.
void sssp_landmark_bounds(sg_ctx* ctx, const SsspDevPlan& p, uint32_t n_used, uint32_t row_begin,
                          const uint64_t* out_lat, const uint32_t* sat_row, int kb);

}  // namespace sg
