// sg_deliver.hip -- one scheduling round of inter-host packet delivery.
//
// Replaces the per-packet body of Worker::send_packet (worker.rs:322-397) and
// WorkerShared::push_packet_to_host (worker.rs:597-607), batched at the round
// boundary.  Batching is exact: every packet sent in [start, end) is delivered
// at max(now + latency, end) (worker.rs:380-384) and Host::execute(end) only
// pops events < end (host.rs:749-758), so no destination can observe a packet
// of this round before the round ends.
//
// Pipeline (all on the context stream, no fills or copies):
//   k_host_off        per packet: host CSR host_off[h], grouping check
//   k_walk            block per 64 source hosts: resolve dst (Dns::addr_to_host_id),
//                     path cell, Xoshiro256++ f64 draw, drop test, arrival time,
//                     event id -- the host's packets in send order
//   k_reduce_stats    round minima + error flags -> pinned host-mapped block
//   k_sb_scatter      delivered packets -> runs in fixed super-bucket regions
//   k_sb_sort_region  block per super-bucket: dst_offsets, EventQueue order per
//                     destination (rank sort; LDS bitonic for big ones)
//   scan-path fallback (a hot destination overfills a region): k_sb_hist, scan,
//   k_sb_scatter (exact positions), k_sb_sort, k_sort_big.
// Event order (event.rs:84-155): (time, Packet < Local, src_host_id,
// src_host_event_id).  Inside a bucket every element is a packet; since the
// input is grouped by ascending source host in send order and event ids grow
// in send order, (src_host_id, src_host_event_id) order == packet-index order,
// so the bucket key is (deliver_time, packet index).
#include <algorithm>
#include <cstring>
#include <utility>
#include <vector>

#include "sg_device.h"
#include "sg_internal.h"

struct sg_hosts {
  sg_ctx* ctx = nullptr;
  uint32_t n = 0;
  uint32_t* route = nullptr;  // host -> routing-table index
  uint64_t* rng = nullptr;    // SoA [4][n]
  uint64_t* ctr = nullptr;    // n
  // address -> (host, routing index): dense window or sorted table (the pair
  // in one 8-byte entry, so resolving a destination is one dependent load)
  uint32_t ip_base = 0, dense_span = 0;
  uint2* dense = nullptr;
  uint32_t* sorted_ip = nullptr;
  uint2* sorted_host = nullptr;
  uint32_t max_route = 0;  // largest routing-table index of any host
  uint32_t min_route = 0;  // smallest (with max_route: a table shard holding every host's row needs no per-round check)
  ~sg_hosts() {
    void* ps[] = {route, rng, ctr, dense, sorted_ip, sorted_host};
    for (void* p : ps)
      if (p) (void)hipFree(p);
  }
};

namespace sg {

constexpr uint32_t NONE = ~0u;
constexpr int SMALL_BUCKET = 32;
constexpr uint32_t INBLOCK_RANK_SMALL = 32;  // region path: rank sort up to this many entries per slot,
constexpr uint32_t WAVE_SORT_MAX = 256;      // in-wave bitonic sort up to this many, the block's beyond
// (up to 4 keys per lane: 8 took the region sort to 256 VGPRs, one block per CU)
constexpr int SORT_BLOCK = 256;
constexpr int SORT_CHUNK = 2048;  // elements sorted in LDS per chunk

enum : uint32_t { ERR_UNSORTED = 1, ERR_SRC_RANGE = 2, ERR_ROUTE_RANGE = 4, ERR_NOT_LOCAL = 8, ERR_TIME_OVERFLOW = 16 };
// flags that reject a whole batch before any host state changes (raised by k_host_off)
constexpr uint32_t ERR_BATCH = ERR_UNSORTED | ERR_SRC_RANGE | ERR_ROUTE_RANGE;

struct HostMap {
  uint32_t ip_base, dense_span, n_sorted;
  const uint2* dense;
  const uint32_t* sorted_ip;
  const uint2* sorted_host;
  // Dns::addr_to_host_id (dns.rs:174-176): (host, its routing index), host = NONE if unknown
  __device__ __forceinline__ uint2 resolve(uint32_t ip) const {
    if (dense) {
      uint32_t off = ip - ip_base;
      return off < dense_span ? dense[off] : make_uint2(NONE, 0);
    }
    uint32_t lo = 0, hi = n_sorted;
    while (lo < hi) {
      uint32_t mid = (lo + hi) >> 1;
      if (sorted_ip[mid] < ip)
        lo = mid + 1;
      else
        hi = mid;
    }
    return (lo < n_sorted && sorted_ip[lo] == ip) ? sorted_host[lo] : make_uint2(NONE, 0);
  }
};

__global__ void k_seed_hosts(const uint64_t* __restrict__ seed, uint32_t n, uint64_t* __restrict__ rng) {
  for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h < n; h += gridDim.x * blockDim.x) {
    Xoshiro x = xoshiro_seed_from_u64(seed[h]);
    rng[h] = x.s0;
    rng[(size_t)n + h] = x.s1;
    rng[2 * (size_t)n + h] = x.s2;
    rng[3 * (size_t)n + h] = x.s3;
  }
}

// Host CSR over the packets: host_off[h] = first packet whose source is >= h
// (h = 0..H).  Also checks the grouping (ascending source hosts) and, when
// `route` is given, that every sending host's route row lies in the table shard
// [row_begin, row_begin + n_rows): a batch failing either check is rejected by
// the walk before it touches any host's RNG stream or event counter.
__global__ void k_host_off(const uint32_t* __restrict__ src, uint32_t P, uint32_t H,
                           uint32_t* __restrict__ host_off, uint32_t* __restrict__ err,
                           const uint32_t* __restrict__ route = nullptr, uint32_t row_begin = 0,
                           uint32_t n_rows = 0) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i <= P; i += gridDim.x * blockDim.x) {
    const uint32_t s = i < P ? src[i] : H;
    if (s > H || (i < P && s == H)) {
      atomicOr(err, ERR_SRC_RANGE);
      continue;
    }
    const int64_t prev = i ? (int64_t)min(src[i - 1], H) : -1;
    if (prev > (int64_t)s) {
      atomicOr(err, ERR_UNSORTED);
      continue;
    }
    if (route && i < P && (int64_t)s != prev) {  // first packet of host s
      const uint32_t r = route[s];
      if (r < row_begin || r - row_begin >= n_rows) atomicOr(err, ERR_ROUTE_RANGE);
    }
    for (int64_t h = prev + 1; h <= (int64_t)s; h++) host_off[h] = i;
  }
}

// k_host_off with four packets per thread read by one 16-B load (src 16-B
// aligned), the previous packet's source taken from the neighbouring lane:
// the 10M-packet C5 round spent 38 us in the one-packet-per-thread version.
__global__ void __launch_bounds__(256) k_host_off4(const uint32_t* __restrict__ src, uint32_t P, uint32_t H,
                                                   uint32_t* __restrict__ host_off, uint32_t* __restrict__ err,
                                                   const uint32_t* __restrict__ route, uint32_t row_begin,
                                                   uint32_t n_rows) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x, i0 = 4 * t;
  const int lane = threadIdx.x & 63;
  uint32_t v[4];
  if (i0 + 3 < P) {
    const uint4 x = *reinterpret_cast<const uint4*>(src + i0);
    v[0] = x.x;
    v[1] = x.y;
    v[2] = x.z;
    v[3] = x.w;
  } else {
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = i0 + q < P ? src[i0 + q] : H;
  }
  // the source before i0: lane - 1's last one, or a load at a wave's first lane
  uint32_t before = __shfl_up(v[3], 1, 64);
  if (lane == 0) before = i0 ? src[min(i0 - 1, P - 1)] : 0;
  // every packet's route row loaded up front (L2 hits, all four in flight): under the
  // first-packet branch below the compiler waited for each in turn
  uint32_t rr[4] = {0u, 0u, 0u, 0u};
  if (route && H) {
#pragma unroll
    for (int q = 0; q < 4; q++) rr[q] = route[min(v[q], H - 1)];
  }
  if (i0 > P) return;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t i = i0 + q;
    if (i > P) break;
    const uint32_t s = v[q];
    const uint32_t pv = q ? v[q - 1] : before;
    if (s > H || (i < P && s == H)) {
      atomicOr(err, ERR_SRC_RANGE);
      continue;
    }
    const int64_t prev = i ? (int64_t)min(pv, H) : -1;
    if (prev > (int64_t)s) {
      atomicOr(err, ERR_UNSORTED);
      continue;
    }
    if (route && i < P && (int64_t)s != prev) {  // first packet of host s
      const uint32_t r = rr[q];
      if (r < row_begin || r - row_begin >= n_rows) atomicOr(err, ERR_ROUTE_RANGE);
    }
    for (int64_t h = prev + 1; h <= (int64_t)s; h++) host_off[h] = i;
  }
}

struct WalkArgs {
  const uint32_t* src;
  const uint32_t* dst_ip;
  const uint32_t* payload;
  const uint64_t* send;
  const uint32_t* skip;  // sg_packets.rng_skip: other consumers' steps before each packet, or null
  uint32_t P, H;
  const uint32_t* host_off;
  const uint32_t* route;
  uint64_t* rng;
  uint64_t* ctr;
  HostMap map;
  const uint64_t* tab_lat;
  const float* tab_loss;
  const uint64_t* tab_key;  // packed (lat << 32 | bits(loss)) cells, or null
  uint32_t n_cols, row_begin, n_rows;
  uint64_t round_end, sim_end, bootstrap_end;
  uint8_t* status;
  uint64_t* deliver;
  uint64_t* eid;
  uint32_t* dst_host;
  unsigned long long* blk_stats;  // per block: [n_delivered, min_deliver, min_lat] (reduced by k_reduce_stats)
  uint32_t* err;
  unsigned long long* pair_count;  // CNT: per table cell, +1 per delivered packet (sg_ctx_set_packet_counters)
};

// A block owns WALK_HOSTS consecutive source hosts; their packets are one
// contiguous range, processed in chunks of WALK_CHUNK staged in LDS:
//  1. packet-parallel (all threads, coalesced): send time, destination
//     resolution (Dns::addr_to_host_id, worker.rs:341), path gather
//     (latency, loss) -- every independent load in flight at once;
//  2. host-sequential (one lane per host): the host's packets in send order
//     against its Xoshiro256++ stream -- only LDS traffic on the serial chain;
//  3. packet-parallel: coalesced stores of status, arrival time, event id and
//     destination.
constexpr int WALK_THREADS = 256;
constexpr int WALK_HOSTS = 64;
constexpr int WALK_CHUNK = 1024;
enum : uint8_t { W_SIM_END = 0, W_NO_DST = 1, W_DRAW = 2, W_PAYLOAD = 4, W_BOOT = 8 };

// PACKED: the path cell is one (lat << 32 | bits(loss)) word, kept whole in
// LDS (17 B of LDS per staged packet, so every block of a 100k-host round is
// resident at once); else latency and loss are staged separately (21 B).  The
// destination stays in the registers of the thread that resolved it: phases 1
// and 3 map packets to threads identically.
// (the unpacked two-array variant needs 74 VGPRs and stays at 6 waves per SIMD)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wpass-failed"
// SKIP: packets carry rng_skip (sg_packets), staged in LDS beside the rest (4 B
// more per packet: 7 blocks per CU instead of 8, still every block of a 100k-host
// round resident); a batch without it runs the SKIP = false variant unchanged.
// CNT: every delivered packet adds one to its path's cell in a.pair_count
// (RoutingInfo::increment_packet_count, graph/mod.rs:451-459, called from worker.rs:373); a round
// without counters runs CNT = false unchanged.
template <bool PACKED, bool SKIP, bool CNT = false>
// At most 64 VGPRs (8 waves per SIMD, 8 blocks per CU): a 100k-host round's
// 1,563 blocks are then all resident at once.  At 74 VGPRs 6 blocks fit a CU,
// and the last 27 blocks ran as a second round, doubling the kernel time.
__global__ void __launch_bounds__(WALK_THREADS) __attribute__((amdgpu_waves_per_eu(8, 8))) k_walk(WalkArgs a) {
  __shared__ uint64_t s_t[WALK_CHUNK];                  // send time -> arrival time
  __shared__ uint64_t s_l[WALK_CHUNK];                  // path latency (or cell) -> event id
  __shared__ float s_loss[PACKED ? 1 : WALK_CHUNK];     // path packet loss (two-array form)
  __shared__ uint8_t s_f[WALK_CHUNK];                   // W_* flags -> SG_PKT_* status
  __shared__ uint32_t s_skip[SKIP ? WALK_CHUNK : 1];    // other consumers' RNG steps before the packet
  const uint32_t h0 = blockIdx.x * WALK_HOSTS;
  const uint32_t t = threadIdx.x;
  if (*a.err & ERR_BATCH) {
    // rejected batch (k_host_off): no host state changes; every packet's
    // destination slot reads NONE so the bucketing that follows stays in bounds
    for (uint32_t i = blockIdx.x * WALK_THREADS + t; i < a.P; i += gridDim.x * WALK_THREADS) a.dst_host[i] = NONE;
    if (t == 0) {
      a.blk_stats[3 * blockIdx.x] = 0;
      a.blk_stats[3 * blockIdx.x + 1] = ~0ull;
      a.blk_stats[3 * blockIdx.x + 2] = ~0ull;
    }
    return;
  }
  // clamped (defensive: k_host_off wrote every entry of an accepted batch)
  const uint32_t p0 = min(a.host_off[min(h0, a.H)], a.P);
  const uint32_t p1 = max(min(a.host_off[min(h0 + WALK_HOSTS, a.H)], a.P), p0);
  // walker lanes: thread t < WALK_HOSTS walks host h0 + t
  const uint32_t h = h0 + t;
  const bool walker = t < WALK_HOSTS && h < a.H;
  uint32_t hb = 0, he = 0;
  Xoshiro x{0, 0, 0, 0};
  uint64_t c = 0;
  if (walker) {  // the stream state loads issue beside the offsets (off the dependent chain)
    hb = min(a.host_off[h], a.P);
    he = max(min(a.host_off[h + 1], a.P), hb);
    x = Xoshiro{a.rng[h], a.rng[(size_t)a.H + h], a.rng[2 * (size_t)a.H + h], a.rng[3 * (size_t)a.H + h]};
    c = a.ctr[h];
  }
  unsigned long long nd = 0, mind = ~0ull, minl = ~0ull;
  for (uint32_t c0 = p0; c0 < p1; c0 += WALK_CHUNK) {
    const uint32_t c1 = min(c0 + WALK_CHUNK, p1);
    // 1. packet-parallel gather, PPT packets per thread batched level by level
    //    (inputs; address map -> (destination, its route column) and the
    //    source's route row; path cell), so a thread has three dependent round
    //    trips per chunk
    constexpr int PPT = WALK_CHUNK / WALK_THREADS;
    uint64_t now[PPT];
    uint32_t ip[PPT], sh[PPT], d[PPT], r[PPT];
    uint8_t f[PPT];
    uint32_t sk[PPT];
    size_t cellq[CNT ? PPT : 1];  // CNT: the path's cell, for the counter
#pragma unroll
    for (int q = 0; q < PPT; q++) {
      const uint32_t i = min(c0 + t + q * WALK_THREADS, c1 - 1);
      sk[q] = SKIP ? a.skip[i] : 0u;
      now[q] = a.send[i];
      ip[q] = a.dst_ip[i];
      sh[q] = a.src[i];
      f[q] = a.payload[i] > 0 ? W_PAYLOAD : 0;
    }
    // Loads below are branch-free where the map is a dense window (the usual
    // case; a uniform branch): a lane with nothing to read reads entry 0 and
    // drops it.  Under per-lane branches the compiler waited for each load
    // before issuing the next one, so the PPT packets' round trips ran in turn.
    if (a.map.dense) {
#pragma unroll
      for (int q = 0; q < PPT; q++) {
        if (now[q] < a.bootstrap_end) f[q] |= W_BOOT;
        const uint32_t off = ip[q] - a.map.ip_base;
        const bool ok = now[q] < a.sim_end && off < a.map.dense_span;  // worker.rs:332-335, 341
        const uint2 v = a.map.dense[ok ? off : 0];
        d[q] = ok ? v.x : NONE;
        ip[q] = ok ? v.y : 0;  // reuse: the destination's route column
        r[q] = a.route[min(sh[q], a.H - 1)];  // sh < H in an accepted batch
      }
    } else {
#pragma unroll
      for (int q = 0; q < PPT; q++) {
        if (now[q] < a.bootstrap_end) f[q] |= W_BOOT;
        const uint2 hr = now[q] < a.sim_end ? a.map.resolve(ip[q]) : make_uint2(NONE, 0);  // worker.rs:332-335, 341
        d[q] = hr.x;
        ip[q] = hr.y;  // reuse: the destination's route column
        r[q] = a.route[min(sh[q], a.H - 1)];  // sh < H in an accepted batch
      }
    }
#pragma unroll
    for (int q = 0; q < PPT; q++) {
      const bool past_end = !(now[q] < a.sim_end);
      if (!past_end && d[q] == NONE) f[q] |= W_NO_DST;
      if (d[q] != NONE && (r[q] < a.row_begin || r[q] - a.row_begin >= a.n_rows)) {
        atomicOr(a.err, ERR_ROUTE_RANGE);
        f[q] |= W_NO_DST;
        d[q] = NONE;
      }
    }
#pragma unroll
    for (int q = 0; q < PPT; q++) {
      const uint32_t i = c0 + t + q * WALK_THREADS;
      uint64_t lat = 0;  // PACKED: the whole cell
      float loss = 0.0f;
      const bool ok = d[q] != NONE;  // then the table has cells (a destination needs its route column)
      const size_t cell = ok ? (size_t)(r[q] - a.row_begin) * a.n_cols + ip[q] : 0;
      if constexpr (CNT) cellq[q] = cell;
      if (a.n_cols && a.n_rows) {  // uniform; branch-free gathers (cell 0 for the lanes that drop them)
        if (PACKED) {
          lat = a.tab_key[cell];  // one 8-byte gather
        } else {
          lat = a.tab_lat[cell];
          loss = a.tab_loss[cell];
        }
      }
      if (ok) f[q] |= W_DRAW;
      if (i < c1) {
        const uint32_t k = i - c0;
        s_t[k] = now[q];
        s_l[k] = lat;
        if (!PACKED) s_loss[k] = loss;
        s_f[k] = f[q];
        if (SKIP) s_skip[k] = sk[q];
      }
    }
    __syncthreads();
    // 2. host-sequential walk (worker.rs:326-397)
    if (walker) {
      const uint32_t b = max(hb, c0), e = min(he, c1);
      for (uint32_t i = b; i < e; i++) {
        const uint32_t k = i - c0;
        const uint8_t f = s_f[k];
        if (SKIP)  // the steps Host::random_mut()'s other consumers took before this send (sg_packets.rng_skip)
          for (uint32_t z = s_skip[k]; z; z--) (void)x.next_u64();
        uint8_t st;
        uint64_t arr = 0, id = ~0ull;
        if (f & W_DRAW) {
          const uint64_t cell = s_l[k];
          const float loss = PACKED ? __uint_as_float((uint32_t)cell) : s_loss[k];
          const uint64_t lat = PACKED ? cell >> 32 : cell;
          // reliability = f64::from(1.0f32 - loss) (worker.rs:357-359, 526-531)
          const double rel = (double)__fsub_rn(1.0f, loss);
          const double chance = x.next_f64();  // worker.rs:360
          if (!(f & W_BOOT) && chance >= rel && (f & W_PAYLOAD)) {  // worker.rs:365-368
            st = SG_PKT_DROP_LOSS;
          } else {
            arr = s_t[k] + lat;  // worker.rs:381; EmulatedTime + SimulationTime panics past EMUTIME_MAX
            if (arr < lat || arr == ~0ull) {  // (emulated_time.rs:121-126): a failed call here
              atomicOr(a.err, ERR_TIME_OVERFLOW);
              arr = ~0ull - 1;
            }
            if (arr < a.round_end) arr = a.round_end;  // worker.rs:381-384
            id = c++;                                  // host.rs:649-653
            st = SG_PKT_DELIVERED;
            nd++;
            mind = min(mind, (unsigned long long)arr);
            minl = min(minl, (unsigned long long)lat);
          }
        } else {
          st = (f & W_NO_DST) ? SG_PKT_DROP_NO_DST : SG_PKT_SIM_END;
        }
        s_t[k] = arr;
        s_l[k] = id;
        s_f[k] = st;
      }
    }
    __syncthreads();
    // 3. coalesced stores (the same packet -> thread map as phase 1)
#pragma unroll
    for (int q = 0; q < PPT; q++) {
      const uint32_t i = c0 + t + q * WALK_THREADS;
      if (i < c1) {
        const uint32_t k = i - c0;
        const uint8_t st = s_f[k];
        a.status[i] = st;
        a.deliver[i] = s_t[k];
        a.eid[i] = s_l[k];
        a.dst_host[i] = st == SG_PKT_DELIVERED ? d[q] : NONE;
        if constexpr (CNT)  // u64: saturation (the reference's saturating_add) is out of reach
          if (st == SG_PKT_DELIVERED) atomicAdd(&a.pair_count[cellq[q]], 1ull);
      }
    }
    __syncthreads();
  }
  if (walker && hb < he) {
    a.rng[h] = x.s0;
    a.rng[(size_t)a.H + h] = x.s1;
    a.rng[2 * (size_t)a.H + h] = x.s2;
    a.rng[3 * (size_t)a.H + h] = x.s3;
    a.ctr[h] = c;
  }
  if (t < 64) {  // the walkers are wave 0
    for (int dd = 32; dd > 0; dd >>= 1) {
      nd += __shfl_xor(nd, dd, 64);
      mind = min(mind, (unsigned long long)__shfl_xor(mind, dd, 64));
      minl = min(minl, (unsigned long long)__shfl_xor(minl, dd, 64));
    }
    // plain per-block stores: thousands of same-address atomics serialise at the memory
    if (t == 0) {
      a.blk_stats[3 * blockIdx.x] = nd;
      a.blk_stats[3 * blockIdx.x + 1] = mind;
      a.blk_stats[3 * blockIdx.x + 2] = minl;
    }
  }
}
#pragma clang diagnostic pop

// Round statistics: sum / min / min over the walk blocks' partials, written
// with the source phase's error flags straight into the context's pinned
// host-mapped return block.  Clears the flags (for the next round) and the
// big-slot counter (for this round's bucketing, which runs next).  One block:
// k_reduce_stats, or the extra block of the region scatter (StatsJob).
struct StatsJob {
  const unsigned long long* blk;  // null: nothing to reduce
  uint32_t n;
  uint32_t* err;
  uint32_t* big_count;
  sg_round_ret* ret;
  unsigned long long* row;  // optional (device): the stats also go to row[0..2] (padded exchange)
};

template <int NT>
__device__ __forceinline__ void reduce_stats_block(const StatsJob& j) {
  __shared__ unsigned long long r[3][NT / 64];
  unsigned long long nd = 0, mind = ~0ull, minl = ~0ull;
  for (uint32_t i = threadIdx.x; i < j.n; i += NT) {
    nd += j.blk[3 * i];
    mind = min(mind, j.blk[3 * i + 1]);
    minl = min(minl, j.blk[3 * i + 2]);
  }
  for (int d = 32; d > 0; d >>= 1) {
    nd += __shfl_xor(nd, d, 64);
    mind = min(mind, (unsigned long long)__shfl_xor(mind, d, 64));
    minl = min(minl, (unsigned long long)__shfl_xor(minl, d, 64));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    r[0][w] = nd;
    r[1][w] = mind;
    r[2][w] = minl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < NT / 64; i++) {
      nd += r[0][i];
      mind = min(mind, r[1][i]);
      minl = min(minl, r[2][i]);
    }
    j.ret->stats[0] = nd;
    j.ret->stats[1] = mind;
    j.ret->stats[2] = minl;
    if (j.row) {
      j.row[0] = nd;
      j.row[1] = mind;
      j.row[2] = minl;
    }
    j.ret->err = *j.err;
    *j.err = 0;
    *j.big_count = 0;
  }
}

__global__ void __launch_bounds__(1024) k_reduce_stats(StatsJob j) { reduce_stats_block<1024>(j); }

__device__ __forceinline__ bool key_less(uint64_t ta, uint64_t ka, uint64_t tb, uint64_t kb) {
  return ta < tb || (ta == tb && ka < kb);
}

// Block per large bucket.  Chunks of SORT_CHUNK are bitonic-sorted in LDS,
// then merged pairwise (merge path) between two global buffers.
__global__ void __launch_bounds__(SORT_BLOCK)
    k_sort_big(const uint32_t* __restrict__ off, const uint32_t* __restrict__ big_list,
               const uint32_t* __restrict__ big_count, uint64_t* __restrict__ kt,
               uint64_t* __restrict__ kk, uint32_t* __restrict__ ki, uint64_t* __restrict__ kt2,
               uint64_t* __restrict__ kk2, uint32_t* __restrict__ ki2, uint32_t* __restrict__ order) {
  __shared__ uint64_t st[SORT_CHUNK];
  __shared__ uint64_t sk[SORT_CHUNK];
  __shared__ uint32_t si[SORT_CHUNK];
  const uint32_t nbig = *big_count;
  for (uint32_t q = blockIdx.x; q < nbig; q += gridDim.x) {
    const uint32_t h = big_list[q];
    const uint32_t b = off[h], e = off[h + 1], n = e - b;
    // 1. sort chunks in LDS
    for (uint32_t c0 = 0; c0 < n; c0 += SORT_CHUNK) {
      const uint32_t cn = min((uint32_t)SORT_CHUNK, n - c0);
      uint32_t pow2 = 1;
      while (pow2 < cn) pow2 <<= 1;
      for (uint32_t i = threadIdx.x; i < pow2; i += SORT_BLOCK) {
        const bool in = i < cn;
        st[i] = in ? kt[b + c0 + i] : ~0ull;
        sk[i] = in ? kk[b + c0 + i] : ~0ull;
        si[i] = in ? ki[b + c0 + i] : ~0u;
      }
      __syncthreads();
      for (uint32_t k = 2; k <= pow2; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
          for (uint32_t i = threadIdx.x; i < pow2; i += SORT_BLOCK) {
            uint32_t l = i ^ j;
            if (l > i) {
              bool up = (i & k) == 0;
              bool sw = up ? key_less(st[l], sk[l], st[i], sk[i]) : key_less(st[i], sk[i], st[l], sk[l]);
              if (sw) {
                uint64_t tt = st[i];
                st[i] = st[l];
                st[l] = tt;
                uint64_t tk = sk[i];
                sk[i] = sk[l];
                sk[l] = tk;
                uint32_t ii = si[i];
                si[i] = si[l];
                si[l] = ii;
              }
            }
          }
          __syncthreads();
        }
      }
      for (uint32_t i = threadIdx.x; i < cn; i += SORT_BLOCK) {
        kt[b + c0 + i] = st[i];
        kk[b + c0 + i] = sk[i];
        ki[b + c0 + i] = si[i];
      }
      __syncthreads();
    }
    // 2. merge runs of width w into the other buffer until one run remains
    uint64_t *at = kt + b, *ak = kk + b, *bt = kt2 + b, *bk = kk2 + b;
    uint32_t *ai = ki + b, *bi = ki2 + b;
    for (uint32_t w = SORT_CHUNK; w < n; w <<= 1) {
      for (uint32_t p = threadIdx.x; p < n; p += SORT_BLOCK) {
        const uint32_t s = (p / (2 * w)) * (2 * w);  // first run of the pair holding output p
        const uint32_t m = min(s + w, n), t = min(s + 2 * w, n);
        const uint32_t k = p - s;  // rank within the merged pair
        // merge path: i elements from run A (s..m), k - i from run B (m..t)
        uint32_t lo = k > (t - m) ? k - (t - m) : 0, hi = min(k, m - s);
        while (lo < hi) {
          uint32_t i = (lo + hi) >> 1;
          uint32_t j = k - i;
          if (key_less(at[s + i], ak[s + i], at[m + j - 1], ak[m + j - 1]))
            lo = i + 1;
          else
            hi = i;
        }
        const uint32_t i = lo, j = k - lo;
        bool takeA;
        if (s + i >= m)
          takeA = false;
        else if (m + j >= t)
          takeA = true;
        else
          takeA = !key_less(at[m + j], ak[m + j], at[s + i], ak[s + i]);
        const uint32_t src = takeA ? s + i : m + j;
        bt[p] = at[src];
        bk[p] = ak[src];
        bi[p] = ai[src];
      }
      __syncthreads();
      uint64_t* t0 = at;
      at = bt;
      bt = t0;
      uint64_t* k0 = ak;
      ak = bk;
      bk = k0;
      uint32_t* i0 = ai;
      ai = bi;
      bi = i0;
    }
    for (uint32_t p = threadIdx.x; p < n; p += SORT_BLOCK) order[b + p] = ai[p];
    __syncthreads();
  }
}

// ---- sharded delivery: pack delivered records by destination owner --------
constexpr int PACK_BLOCK = 256;
constexpr uint32_t MAX_RANKS = 64;

__global__ void __launch_bounds__(PACK_BLOCK)
    k_owner_count(const uint32_t* __restrict__ dst_host, uint32_t P, const uint32_t* __restrict__ owner,
                  uint32_t n_ranks, uint32_t* __restrict__ block_counts) {
  __shared__ uint32_t cnt[MAX_RANKS];
  for (uint32_t r = threadIdx.x; r < n_ranks; r += PACK_BLOCK) cnt[r] = 0;
  __syncthreads();
  const uint32_t chunk = (P + gridDim.x - 1) / gridDim.x;
  const uint32_t i0 = blockIdx.x * chunk, i1 = min(P, i0 + chunk);
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += PACK_BLOCK) {
    uint32_t d = dst_host[i];
    if (d != NONE) atomicAdd(&cnt[owner[d]], 1u);
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < n_ranks; r += PACK_BLOCK) block_counts[r * gridDim.x + blockIdx.x] = cnt[r];
}

// padded (optional): rank r's k-th record goes to padded[r * cap + k] when k < cap
// (the fixed-split exchange), and to send[p] (its compact position) otherwise.
__global__ void __launch_bounds__(PACK_BLOCK)
    k_owner_scatter(const uint32_t* __restrict__ src_host, const uint32_t* __restrict__ dst_host,
                    const uint64_t* __restrict__ deliver, const uint64_t* __restrict__ eid,
                    const uint64_t* __restrict__ ctr_start, uint32_t P, const uint32_t* __restrict__ owner,
                    uint32_t n_ranks, const uint32_t* __restrict__ block_off, sg_record* __restrict__ send,
                    sg_record* __restrict__ padded, uint32_t cap) {
  __shared__ uint32_t cur[MAX_RANKS], start[MAX_RANKS];
  for (uint32_t r = threadIdx.x; r < n_ranks; r += PACK_BLOCK) {
    cur[r] = block_off[r * gridDim.x + blockIdx.x];
    start[r] = block_off[r * gridDim.x];
  }
  __syncthreads();
  const uint32_t chunk = (P + gridDim.x - 1) / gridDim.x;
  const uint32_t i0 = blockIdx.x * chunk, i1 = min(P, i0 + chunk);
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += PACK_BLOCK) {
    uint32_t d = dst_host[i];
    if (d == NONE) continue;
    const uint32_t o = owner[d];
    const uint32_t p = atomicAdd(&cur[o], 1u);
    uint32_t s = src_host[i];
    sg_record r;
    r.deliver_time_ns = deliver[i];
    r.order_key = ((uint64_t)s << 32) | (uint32_t)(eid[i] - ctr_start[s]);
    r.event_id = eid[i];
    r.packet = i;
    r.dst_host = d;
    const uint32_t k = p - start[o];
    if (padded && k < cap)
      padded[(size_t)o * cap + k] = r;
    else
      send[p] = r;
  }
}

// xrow[3 + r] = records this rank sends rank r (block_off: exclusive scan of the
// (rank, block) counts, nb blocks per rank).
__global__ void k_xrow_counts(const uint32_t* __restrict__ block_off, uint32_t nb, uint32_t n_ranks,
                              unsigned long long* __restrict__ xrow) {
  const uint32_t r = threadIdx.x;
  if (r < n_ranks) xrow[3 + r] = block_off[(size_t)(r + 1) * nb] - block_off[(size_t)r * nb];
}

// The fixed-split exchange's fallback: every record of `padded` to its compact position.
__global__ void k_pad_to_compact(const sg_record* __restrict__ padded, uint32_t cap,
                                 const unsigned long long* __restrict__ xrow, uint32_t n_ranks,
                                 sg_record* __restrict__ compact) {
  __shared__ uint32_t start[MAX_RANKS + 1];
  if (threadIdx.x == 0) {
    uint32_t a = 0;
    for (uint32_t r = 0; r < n_ranks; r++) {
      start[r] = a;
      a += (uint32_t)xrow[3 + r];
    }
  }
  __syncthreads();
  const size_t total = (size_t)n_ranks * cap;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const uint32_t r = (uint32_t)(e / cap), k = (uint32_t)(e - (size_t)r * cap);
    if (k < min((uint32_t)xrow[3 + r], cap)) compact[start[r] + k] = padded[e];
  }
}

// After the bucketing of a padded exchange: the round's global stats (sum, min,
// min over the gathered rows), this rank's receive counts and the largest pair
// count, into the mapped return block; the bucketing's error word joins the
// source phase's flags there.
__global__ void k_xall_reduce(const unsigned long long* __restrict__ xall, uint32_t n_ranks, uint32_t rank,
                              uint32_t* __restrict__ err, sg_round_ret* ret) {
  const uint32_t b = threadIdx.x, w = 3 + n_ranks;
  const bool on = b < n_ranks;
  unsigned long long nd = on ? xall[(size_t)b * w] : 0, md = on ? xall[(size_t)b * w + 1] : ~0ull,
                     ml = on ? xall[(size_t)b * w + 2] : ~0ull, pm = 0;
  if (on) {
    for (uint32_t r = 0; r < n_ranks; r++) pm = max(pm, xall[(size_t)b * w + 3 + r]);
    ret->recv_cnt[b] = (uint32_t)xall[(size_t)b * w + 3 + rank];
  }
  for (int d = 32; d > 0; d >>= 1) {
    nd += __shfl_xor(nd, d, 64);
    md = min(md, (unsigned long long)__shfl_xor(md, d, 64));
    ml = min(ml, (unsigned long long)__shfl_xor(ml, d, 64));
    pm = max(pm, (unsigned long long)__shfl_xor(pm, d, 64));
  }
  if (b == 0) {
    ret->stats[0] = nd;
    ret->stats[1] = md;
    ret->stats[2] = ml;
    ret->pair_max = (uint32_t)min(pm, 0xFFFFFFFFull);
    ret->err |= *err;
    *err = 0;
  }
}

static void fail_flags(uint32_t err) {
  if (err & ERR_SRC_RANGE) throw Error(SG_ERR_INVALID_ARG, "packet source host out of range");
  if (err & ERR_UNSORTED)
    throw Error(SG_ERR_UNSORTED, "packets must be grouped by ascending source host (send order within a host)");
  if (err & ERR_ROUTE_RANGE)
    throw Error(SG_ERR_INVALID_ARG, "a sending host's route row is outside the table shard");
  if (err & ERR_TIME_OVERFLOW)
    throw Error(SG_ERR_TIME_OVERFLOW,
                "send time + path latency overflows EmulatedTime (the reference panics, emulated_time.rs:121-126); "
                "host RNG streams and event counters are not restored");
  if (err & ERR_NOT_LOCAL)
    throw Error(SG_ERR_INVALID_ARG, "a received record's destination host is not local to this rank");
}

// ---------------------------------------------------------------------------
// Destination bucketing without global atomics.
//
// Entries (a delivered packet, or a received record) carry a destination slot
// d, an arrival time t, an order key kk and a value ki.  Result: offsets[d] and
// order[] = the ki of every entry sorted by (d, t, kk) -- EventQueue order per
// destination (event.rs:84-155).
//   1. k_sb_hist    tiles of SB_TILE entries: LDS histogram over super-buckets
//                   (sb = d / spb, a contiguous range of spb slots, sized so a
//                   super-bucket's entries fit one sort block's LDS);
//   2. scan         of the (super-bucket, tile) counts;
//   3. k_sb_scatter entries to their super-bucket (LDS cursors; order inside a
//                   super-bucket is irrelevant, step 4 sorts it fully);
//   4. k_sb_sort    block per super-bucket: per-slot counts and offsets in
//                   LDS, placement by slot, rank sort of each slot by
//                   (t, kk); slots above SMALL_BUCKET entries go to k_sort_big.
// ---------------------------------------------------------------------------
constexpr int SB_THREADS = 256;
constexpr int SB_TILE = 4096;        // entries per hist / scatter block
constexpr int SB_MAX = 4096;         // super-buckets (LDS histogram bins)
constexpr uint32_t CB_MAX = 256;     // coarse buckets of a two-level scatter (and super-buckets per coarse bucket)
static_assert(SB_SUB * SB_MAX + 1 == SB_CTL_STRIDE, "region counters: SB_SUB x SB_MAX counts + the overflow flag");
constexpr uint32_t SB_FLAG = SB_SUB * SB_MAX;  // overflow flag word
constexpr int SB_SLOTS_MAX = 1024;   // slots per super-bucket
// entries a super-bucket sorts in LDS, and the mean entries per super-bucket
// aimed for: 14 B of LDS per entry without a separate order key, 22 B with one
template <bool KK> constexpr int SB_CAP = KK ? 3072 : 4096;
template <bool KK> constexpr int SB_TARGET = KK ? 2048 : 2560;

// Super-bucket of slot d: d / spb as a multiply-high (exact for d < 2^24,
// spb < 2^16: magic = ceil(2^40 / spb)).
struct SbMap {
  uint64_t magic;
  uint32_t spb;
  __device__ __forceinline__ uint32_t of(uint32_t d) const { return (uint32_t)(((uint64_t)d * magic) >> 40); }
};
constexpr int SBT_THREADS = 512;     // k_sb_sort block

struct PacketEntries {  // single GPU: entries are the round's packets, kk = ki = packet index
  static constexpr bool KK = false;  // the order key is the value itself
  static constexpr bool COARSE = false;
  const uint32_t* dst;
  const uint64_t* t;
  __device__ __forceinline__ uint32_t slot(uint32_t e) const { return dst[e]; }
  __device__ __forceinline__ void get(uint32_t e, uint64_t& tt, uint64_t& kk, uint32_t& ki) const {
    tt = t[e];
    kk = e;
    ki = e;
  }
};

struct RecordEntries {  // sharded: entries are received records, slot = the destination's local index
  static constexpr bool KK = true;
  static constexpr bool COARSE = false;
  const sg_record* rec;
  const uint32_t* local;
  uint32_t H;
  uint32_t* err;
  __device__ __forceinline__ uint32_t slot(uint32_t e) const {
    const uint32_t d = rec[e].dst_host;
    const uint32_t s = d < H ? local[d] : NONE;
    if (s == NONE) atomicOr(err, ERR_NOT_LOCAL);
    return s;
  }
  __device__ __forceinline__ void get(uint32_t e, uint64_t& tt, uint64_t& kk, uint32_t& ki) const {
    tt = rec[e].deliver_time_ns;
    kk = rec[e].order_key;
    ki = e;
  }
};

// sharded, fixed-split exchange: block b of `cap` records came from rank b, of which
// the first min(xall[b][3 + rank], cap) are real; the rest are holes (slot NONE)
struct PaddedRecordEntries {
  static constexpr bool KK = true;
  static constexpr bool COARSE = false;
  const sg_record* rec;
  const uint32_t* local;
  uint32_t H;
  uint32_t* err;
  uint32_t cap, w, rank;  // w = 3 + n_ranks (an xall row)
  const unsigned long long* xall;
  __device__ __forceinline__ uint32_t slot(uint32_t e) const {
    const uint32_t b = e / cap, k = e - b * cap;
    if ((unsigned long long)k >= xall[(size_t)b * w + 3 + rank]) return NONE;
    const uint32_t d = rec[e].dst_host;
    const uint32_t s = d < H ? local[d] : NONE;
    if (s == NONE) atomicOr(err, ERR_NOT_LOCAL);
    return s;
  }
  __device__ __forceinline__ void get(uint32_t e, uint64_t& tt, uint64_t& kk, uint32_t& ki) const {
    tt = rec[e].deliver_time_ns;
    kk = rec[e].order_key;
    ki = e;
  }
};

// Second level of a two-level scatter: the entries are the coarse level's runs,
// region `region` per coarse bucket, split into SB_SUB sub-regions whose fill
// counts are in ctl (k_sb_scatter<.., true> with a coarse SbMap).  Entries past
// a sub-region's fill are holes (slot NONE).  ctl_next: the other coarse parity,
// cleared by this level for the next two-level call.
template <bool KK_>
struct CoarseEntries {
  static constexpr bool KK = KK_;
  static constexpr bool COARSE = true;
  const uint32_t* rd;
  const uint64_t* rt;
  const uint64_t* rk;
  const uint32_t* ri;
  const uint32_t* ctl;
  uint32_t* ctl_next;
  uint32_t region, subcap, cpb;  // coarse region, its sub-regions, super-buckets per coarse bucket
  __device__ __forceinline__ uint32_t fill_of(uint32_t e, uint32_t& off, uint32_t& sub) const {
    const uint32_t c = e / region, r = e - c * region;
    sub = r / subcap;
    off = r - sub * subcap;
    return ctl[sub * SB_MAX + c];
  }
  // the kernel stops each tile at its sub-region's fill (fill_of), so every entry asked for is a real one
  __device__ __forceinline__ uint32_t slot(uint32_t e) const { return rd[e]; }
  __device__ __forceinline__ void get(uint32_t e, uint64_t& tt, uint64_t& kk, uint32_t& ki) const {
    tt = rt[e];
    ki = ri[e];
    kk = KK ? rk[e] : (uint64_t)ki;
  }
};

template <class E>
__global__ void __launch_bounds__(SB_THREADS)
    k_sb_hist(E src, uint32_t n, SbMap sm, uint32_t n_sb, uint32_t* __restrict__ tile_hist) {
  __shared__ uint32_t h[SB_MAX];
  for (uint32_t i = threadIdx.x; i < n_sb; i += SB_THREADS) h[i] = 0;
  __syncthreads();
  const uint32_t e0 = blockIdx.x * SB_TILE, e1 = min(e0 + SB_TILE, n);
  for (uint32_t e = e0 + threadIdx.x; e < e1; e += SB_THREADS) {
    const uint32_t d = src.slot(e);
    if (d != NONE) atomicAdd(&h[sm.of(d)], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n_sb; i += SB_THREADS) tile_hist[(size_t)i * gridDim.x + blockIdx.x] = h[i];
}

// Exclusive scan of a[0..n) in LDS by the whole block (NT threads, n <= NT * PER);
// returns the total.  Ends with a barrier.
template <int NT, int PER>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t* a, uint32_t n, uint32_t* wsum) {
  const uint32_t j0 = threadIdx.x * PER;
  uint32_t v[PER], sum = 0;
#pragma unroll
  for (int q = 0; q < PER; q++) {
    v[q] = j0 + q < n ? a[j0 + q] : 0;
    sum += v[q];
  }
  uint32_t incl = sum;
  const int lane = threadIdx.x & 63;
  for (int dd = 1; dd < 64; dd <<= 1) {
    const uint32_t y = __shfl_up(incl, dd, 64);
    if (lane >= dd) incl += y;
  }
  if (lane == 63) wsum[threadIdx.x >> 6] = incl;
  __syncthreads();
  uint32_t base = 0, total = 0;
  for (int w = 0; w < NT / 64; w++) {
    if (w < (int)(threadIdx.x >> 6)) base += wsum[w];
    total += wsum[w];
  }
  uint32_t run = base + incl - sum;
#pragma unroll
  for (int q = 0; q < PER; q++)
    if (j0 + q < n) {
      a[j0 + q] = run;
      run += v[q];
    }
  __syncthreads();
  return total;
}

// Tile -> super-buckets.  The tile is first counting-sorted by super-bucket in
// LDS, so each super-bucket's entries of the tile leave as one contiguous run
// (coalesced stores instead of one scattered store per entry and array).
// REGION: instead of the (super-bucket, tile) scan, a tile claims each run in
// its super-bucket's fixed region of `region` entries with one atomic per
// (tile, super-bucket).  The region is split into SB_SUB sub-regions, one per
// XCD (blockIdx % 8 under round-robin dispatch), each with its own counter, so
// a counter sees an eighth of the tiles' atomics.  A run that would overflow
// its sub-region is dropped and flagged in ctl[SB_FLAG] (the host then reruns
// the scan path).
constexpr int SBS_THREADS = 512;
constexpr uint32_t RUN_DROPPED = 0xFFFFFFFFu;  // cannot be a valid run base (see below)
// NB: the most buckets a call may have (SB_MAX, or CB_MAX for the levels of a
// two-level scatter, whose smaller LDS arrays let two blocks share a CU).
template <class E, bool REGION, uint32_t NB = SB_MAX>
__global__ void __launch_bounds__(SBS_THREADS)
    k_sb_scatter(E src, uint32_t n, SbMap sm, uint32_t n_sb, const uint32_t* __restrict__ tile_off,
                 uint32_t* __restrict__ ctl, uint32_t region, uint32_t* __restrict__ rd, uint64_t* __restrict__ rt,
                 uint64_t* __restrict__ rk, uint32_t* __restrict__ ri, StatsJob stats) {
  if (stats.blk && blockIdx.x == gridDim.x - 1) {  // the extra block: the round's stats (saves a launch)
    reduce_stats_block<SBS_THREADS>(stats);
    return;
  }
  // second level: the coarse level's next-parity counters are zeroed on the way out,
  // after this block's loads and run claims (stores ahead of them made each wait)
  auto zero_next = [&]() {
    if constexpr (E::COARSE)
      for (uint32_t i = blockIdx.x * SBS_THREADS + threadIdx.x; i < SB_CTL_STRIDE; i += gridDim.x * SBS_THREADS)
        src.ctl_next[i] = 0;
  };
  if constexpr (E::COARSE) {
    if (src.ctl[SB_FLAG]) {  // the coarse level overflowed: so does this one (the host reruns the scan path)
      if (blockIdx.x == 0 && threadIdx.x == 0) ctl[SB_FLAG] = 1u;
      zero_next();
      return;
    }
  }
  uint32_t e_lim = n;  // second level: the tile's sub-region holds `fill` entries from its start
  if constexpr (E::COARSE) {
    uint32_t off, sub;  // a tile lies in one sub-region (subcap is a multiple of SB_TILE): skip an empty one
    const uint32_t fill = src.fill_of(blockIdx.x * SB_TILE, off, sub);
    if (off >= fill) {
      zero_next();
      return;
    }
    e_lim = blockIdx.x * SB_TILE + (fill - off);
  }
  // Sub-region of the runs this tile claims.  One level: the tile's XCD (tiles
  // are uniform samples, so each sub-region gets an eighth).  Second level: the
  // coarse sub-region the tile reads, which holds an eighth of its coarse bucket
  // (tile indices would not: a coarse sub-region's full tiles and its partial
  // last tile alternate in parity).
  uint32_t run_sub = blockIdx.x & (SB_SUB - 1);
  // Second level: the tile's entries all lie in one coarse bucket, i.e. in its
  // cpb super-buckets [sb_lo, sb_lo + nsb); local counters cover just those.
  uint32_t sb_lo = 0, nsb = n_sb;
  if constexpr (E::COARSE) {
    uint32_t off;
    src.fill_of(blockIdx.x * SB_TILE, off, run_sub);
    sb_lo = blockIdx.x * SB_TILE / src.region * src.cpb;
    nsb = min(src.cpb, n_sb - sb_lo);
  }
  constexpr int PER = SB_TILE / SBS_THREADS;
  __shared__ uint32_t lcur[NB];   // local start, then cursor
  __shared__ uint32_t lbase[NB];  // global position of the run - local start
  __shared__ uint32_t sd[SB_TILE];
  __shared__ uint64_t st_[SB_TILE];
  __shared__ uint32_t si[SB_TILE];
  __shared__ uint64_t sk[E::KK ? SB_TILE : 1];
  __shared__ uint32_t wsum[SBS_THREADS / 64];
  for (uint32_t i = threadIdx.x; i < nsb; i += SBS_THREADS) lcur[i] = 0;
  __syncthreads();
  const uint32_t e0 = blockIdx.x * SB_TILE, e1 = min(min(e0 + SB_TILE, n), e_lim);
  // every load of the tile up front (one round trip): slot, time, key, value.
  // Branch-free: a lane past the tile's end reads entry e0 again and drops it
  // (conditional loads would each be waited for before the next one issues).
  uint32_t d[PER], vi[PER];
  uint64_t vt[PER], vk[PER];
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t e = e0 + threadIdx.x + k * SBS_THREADS;
    const uint32_t ee = e < e1 ? e : e0;
    const uint32_t dd = src.slot(ee);
    src.get(ee, vt[k], vk[k], vi[k]);
    d[k] = e < e1 ? dd : NONE;
  }
#pragma unroll
  for (int k = 0; k < PER; k++)
    if (d[k] != NONE) atomicAdd(&lcur[sm.of(d[k]) - sb_lo], 1u);
  __syncthreads();
  const uint32_t total = block_exclusive_scan<SBS_THREADS, (NB + SBS_THREADS - 1) / SBS_THREADS>(lcur, nsb, wsum);
  for (uint32_t i = threadIdx.x; i < nsb; i += SBS_THREADS) {
    if (REGION) {
      // the run of super-bucket i: local [lcur[i], lcur[i] + c) -> sub-region slot g..g+c.
      // A kept base is i * region + sub * subcap + g - lcur[i] >= 0 (i = 0: lcur[0] = 0;
      // i > 0: lcur[i] <= SB_TILE <= region), never RUN_DROPPED.
      const uint32_t c = (i + 1 < nsb ? lcur[i + 1] : total) - lcur[i];
      const uint32_t sub = run_sub, subcap = region / SB_SUB;
      uint32_t base = RUN_DROPPED;
      if (c) {
        const uint32_t g = atomicAdd(&ctl[sub * SB_MAX + sb_lo + i], c);
        if (g + c <= subcap)
          base = (sb_lo + i) * region + sub * subcap + g - lcur[i];
        else
          ctl[SB_FLAG] = 1u;
      }
      lbase[i] = base;
    } else {
      lbase[i] = tile_off[(size_t)i * gridDim.x + blockIdx.x] - lcur[i];
    }
  }
  __syncthreads();  // lcur is the cursor from here on
#pragma unroll
  for (int k = 0; k < PER; k++) {
    if (d[k] == NONE) continue;
    const uint32_t p = atomicAdd(&lcur[sm.of(d[k]) - sb_lo], 1u);
    sd[p] = d[k];
    st_[p] = vt[k];
    si[p] = vi[k];
    if (E::KK) sk[p] = vk[k];
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < total; p += SBS_THREADS) {
    const uint32_t dd = sd[p];
    const uint32_t lb = lbase[sm.of(dd) - sb_lo];
    if (REGION && lb == RUN_DROPPED) continue;
    const uint32_t g = lb + p;
    rd[g] = dd;
    rt[g] = st_[p];
    ri[g] = si[p];
    if (E::KK) rk[g] = sk[p];
  }
  zero_next();
}

// Placement of a super-bucket's entries by slot, then per-slot order by (t, kk).
// Without KK the order key is the value (ri) itself.
constexpr uint32_t pow2_ceil(uint32_t x) { return x <= 1 ? 1 : 2 * pow2_ceil((x + 1) / 2); }
static_assert(pow2_ceil(3072) == 4096 && pow2_ceil(4096) == 4096 && pow2_ceil(33) == 64, "pow2_ceil");

// Block-wide bitonic sort of one slot's m entries [b, b + m) of the LDS
// arrays by (t, key), through an index array (idx, >= next pow2 of m
// entries); writes the values in order to out[0..m).
template <bool KK>
__device__ __forceinline__ void slot_bitonic(const uint64_t* Tt, const uint64_t* Tk, const uint32_t* Ti,
                                             uint16_t* idx, uint32_t b, uint32_t m, uint32_t* __restrict__ out) {
  constexpr uint16_t PAD = 0xFFFF;  // sorts last
  uint32_t M = 1;
  while (M < m) M <<= 1;
  for (uint32_t i = threadIdx.x; i < M; i += SBT_THREADS) idx[i] = i < m ? (uint16_t)(b + i) : PAD;
  __syncthreads();
  for (uint32_t k = 2; k <= M; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < M; i += SBT_THREADS) {
        const uint32_t l = i ^ j;
        if (l <= i) continue;
        const uint16_t x = idx[i], y = idx[l];
        // y < x ?
        const bool y_lt_x = x == PAD ? y != PAD
                          : y == PAD ? false
                                     : key_less(Tt[y], KK ? Tk[y] : (uint64_t)Ti[y], Tt[x], KK ? Tk[x] : (uint64_t)Ti[x]);
        if (y_lt_x == ((i & k) == 0)) {
          idx[i] = y;
          idx[l] = x;
        }
      }
      __syncthreads();
    }
  for (uint32_t r = threadIdx.x; r < m; r += SBT_THREADS) out[r] = Ti[idx[r]];
  __syncthreads();
}

// In-wave bitonic sort of one slot's m entries [b, b + m) (m <= 64 R),
// keys in registers: lane l holds elements l, l + 64, ..., l + 64 (R - 1); the
// network's exchanges at distance < 64 are lane shuffles, at 64 and above register
// swaps in the lane.  CK: one compressed u64 key per entry ((t - t_min) << 32 |
// value, unique), the value is its low word.  Else (t, k) pairs and the value
// ride along (k = the record's order key, or the value itself).  Pads (~0) sort
// last: every real key is below ~0 (arrival times stop at EMUTIME_MAX).  No
// barrier: one wave sorts a slot while the block's other waves sort others, where
// the rank sort cost m LDS reads per entry (C5: ~100-entry slots, the round's
// second-largest cost) and the block-wide bitonic a barrier per step.
template <int R, bool KK, bool CK>
__device__ __forceinline__ void wave_sort_slot(const uint64_t* Tt, const uint64_t* Tk, const uint32_t* Ti, uint32_t b,
                                               uint32_t m, uint32_t* __restrict__ out) {
  constexpr uint32_t M = 64u * R;
  const uint32_t lane = threadIdx.x & 63;
  uint64_t t[R], k[R];
  uint32_t v[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint32_t i = lane + 64u * r;
    const bool ok = i < m;
    const uint32_t p = b + (ok ? i : 0u);  // branch-free reads; pads replace the value
    const uint64_t tt = Tt[p];
    const uint32_t vv = Ti[p];
    t[r] = ok ? tt : ~0ull;
    v[r] = vv;
    if constexpr (!CK) {
      const uint64_t kk = KK ? Tk[p] : (uint64_t)vv;
      k[r] = ok ? kk : ~0ull;
    }
  }
  auto less = [&](uint64_t ta, uint64_t ka, uint64_t tb, uint64_t kb) {
    if constexpr (CK) return ta < tb;
    else return ta < tb || (ta == tb && ka < kb);
  };
#pragma unroll
  for (uint32_t kk2 = 2; kk2 <= M; kk2 <<= 1) {
#pragma unroll
    for (uint32_t j = kk2 >> 1; j > 0; j >>= 1) {
      if (j >= 64) {  // partner in this lane's register r ^ (j / 64)
#pragma unroll
        for (int r = 0; r < R; r++) {
          const int r2 = r ^ (int)(j >> 6);
          if (r2 <= r) continue;
          const bool asc = ((lane + 64u * r) & kk2) == 0;
          const bool lt21 = less(t[r2], CK ? 0 : k[r2], t[r], CK ? 0 : k[r]);
          const bool lt12 = less(t[r], CK ? 0 : k[r], t[r2], CK ? 0 : k[r2]);
          if (asc ? lt21 : lt12) {
            const uint64_t xt = t[r];
            t[r] = t[r2];
            t[r2] = xt;
            if constexpr (!CK) {
              const uint64_t xk = k[r];
              k[r] = k[r2];
              k[r2] = xk;
              const uint32_t xv = v[r];
              v[r] = v[r2];
              v[r2] = xv;
            }
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < R; r++) {
          const uint32_t i = lane + 64u * r;
          const uint64_t ot = __shfl_xor((unsigned long long)t[r], (int)j, 64);
          uint64_t ok = 0;
          uint32_t ov = 0;
          if constexpr (!CK) {
            ok = __shfl_xor((unsigned long long)k[r], (int)j, 64);
            ov = __shfl_xor(v[r], (int)j, 64);
          }
          const bool want_min = ((i & j) == 0) == ((i & kk2) == 0);
          const bool o_lt = less(ot, ok, t[r], CK ? 0 : k[r]);
          if (want_min == o_lt) {  // take the partner's element (equal keys: pads, identical)
            t[r] = ot;
            if constexpr (!CK) {
              k[r] = ok;
              v[r] = ov;
            }
          }
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint32_t i = lane + 64u * r;
    if (i < m) out[i] = CK ? (uint32_t)t[r] : v[r];
  }
}

// Per-slot order of a placed super-bucket (slot j = entries [cnt[j], cnt[j+1])
// of Tt/Tk/Ti, Ts = slot per entry): rank sort of small slots; slots above
// SMALL_BUCKET go to k_sort_big (copied to the global kt/kk/ki when placed in
// LDS) or, INBLOCK (LDS only), are bitonic-sorted by this block -- the region
// path, where a super-bucket always fits LDS and no k_sort_big launch is needed.
// CK: Tt holds compressed keys ((t - t_min) << 32 | value), unique per entry, so
// one u64 compare is the (t, kk) order (k_sb_sort_region; single GPU).
template <bool LDS, bool KK, bool INBLOCK, bool CK = false>
__device__ __forceinline__ void slot_orders(uint64_t* Tt, uint64_t* Tk, uint32_t* Ti, uint16_t* Ts, uint32_t s0,
                                            uint32_t ns, uint32_t d0, uint32_t nd, const uint32_t* cnt,
                                            uint64_t* __restrict__ kt, uint64_t* __restrict__ kk,
                                            uint32_t* __restrict__ ki, uint32_t* __restrict__ order,
                                            uint32_t* __restrict__ big_list, uint32_t* __restrict__ big_count) {
  static_assert(LDS || !INBLOCK, "in-block big-slot sort needs the LDS copy");
  // In-block (region path): slots up to INBLOCK_RANK_SMALL entries are rank-sorted,
  // up to WAVE_SORT_MAX sorted by one wave each in registers (a bitonic network whose
  // exchanges below 64 are lane shuffles), larger ones by the whole block.
  constexpr uint32_t SMALL = INBLOCK ? INBLOCK_RANK_SMALL : SMALL_BUCKET;
  constexpr uint32_t MAX_BIG = SB_CAP<KK> / (WAVE_SORT_MAX + 1) + 1;
  constexpr uint32_t MAX_WAVE = SB_CAP<KK> / (SMALL + 1) + 1;
  __shared__ uint32_t n_big, n_wave;
  __shared__ uint16_t bigs[INBLOCK ? MAX_BIG : 1];
  __shared__ uint16_t wslots[INBLOCK ? MAX_WAVE : 1];
  if (INBLOCK && threadIdx.x == 0) {
    n_big = 0;
    n_wave = 0;
  }
  __syncthreads();  // placement complete
  for (uint32_t j = threadIdx.x; j < nd; j += SBT_THREADS) {
    const uint32_t b = cnt[j], e = cnt[j + 1];
    if (e - b > SMALL) {
      if (INBLOCK) {
        if (e - b > WAVE_SORT_MAX)
          bigs[atomicAdd(&n_big, 1u)] = (uint16_t)j;
        else
          wslots[atomicAdd(&n_wave, 1u)] = (uint16_t)j;
        continue;
      }
      big_list[atomicAdd(big_count, 1u)] = d0 + j;
      if (LDS)
        for (uint32_t p = b; p < e; p++) {  // k_sort_big works on the global copy
          kt[s0 + p] = Tt[p];
          kk[s0 + p] = KK ? Tk[p] : (uint64_t)Ti[p];
          ki[s0 + p] = Ti[p];
        }
    }
  }
  // Rank sort inside each small slot: entry p goes to slot start + #(entries of
  // its slot with a smaller (t, kk)); (t, kk) is unique per entry.  One thread
  // per entry, independent LDS reads -- no serial insertion chain.
  for (uint32_t p = threadIdx.x; p < ns; p += SBT_THREADS) {
    const uint32_t j = Ts[p];
    const uint32_t b = cnt[j], e = cnt[j + 1];
    if (e - b > SMALL) continue;  // sorted below / by k_sort_big
    const uint64_t t = Tt[p], k = KK ? Tk[p] : (uint64_t)Ti[p];
    uint32_t rank = 0;
    // 8 entries per step, their LDS reads issued together (one at a time, the
    // loop waited out each read's latency: C5's ~100-entry slots spent most of
    // the sort there)
    uint32_t q = b;
    if constexpr (CK) {  // one compare per entry: the rank sort was VALU-bound on the two-word key_less
      for (; q + 8 <= e; q += 8) {
        uint64_t tq[8];
#pragma unroll
        for (int u = 0; u < 8; u++) tq[u] = Tt[q + u];
#pragma unroll
        for (int u = 0; u < 8; u++) rank += tq[u] < t;
      }
      for (; q < e; q++) rank += Tt[q] < t;
    } else {
      for (; q + 8 <= e; q += 8) {
        uint64_t tq[8], kq[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          tq[u] = Tt[q + u];
          kq[u] = KK ? Tk[q + u] : (uint64_t)Ti[q + u];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) rank += key_less(tq[u], kq[u], t, k);
      }
      for (; q < e; q++) rank += key_less(Tt[q], KK ? Tk[q] : (uint64_t)Ti[q], t, k);
    }
    order[s0 + b + rank] = Ti[p];
  }
  if constexpr (INBLOCK) {
    __syncthreads();  // n_wave is final (it was before the rank sort too; this orders the reads)
    for (uint32_t u = threadIdx.x >> 6; u < n_wave; u += SBT_THREADS / 64) {  // one wave per slot
      const uint32_t j = wslots[u], b = cnt[j], m = cnt[j + 1] - b;
      uint32_t* o = order + s0 + b;
      if (m <= 64)
        wave_sort_slot<1, KK, CK>(Tt, Tk, Ti, b, m, o);
      else if (m <= 128)
        wave_sort_slot<2, KK, CK>(Tt, Tk, Ti, b, m, o);
      else
        wave_sort_slot<4, KK, CK>(Tt, Tk, Ti, b, m, o);
    }
  }
  if (INBLOCK) {
    __syncthreads();  // Ts is free: it becomes the index array
    for (uint32_t u = 0; u < n_big; u++) {
      const uint32_t j = bigs[u], b = cnt[j];
      slot_bitonic<KK>(Tt, Tk, Ti, Ts, b, cnt[j + 1] - b, order + s0 + b);
    }
  }
}

// Placement of a super-bucket's entries by slot (from the global run arrays at
// in0), then slot_orders.  Without KK the order key is the value (ri) itself.
template <bool LDS, bool KK>
__device__ __forceinline__ void sb_place_sort(uint64_t* Tt, uint64_t* Tk, uint32_t* Ti, uint16_t* Ts, uint32_t in0,
                                              uint32_t s0, uint32_t s1, uint32_t d0, uint32_t nd, const uint32_t* cnt,
                                              uint32_t* cur, const uint32_t* __restrict__ rd,
                                              const uint64_t* __restrict__ rt, const uint64_t* __restrict__ rk,
                                              const uint32_t* __restrict__ ri, uint64_t* __restrict__ kt,
                                              uint64_t* __restrict__ kk, uint32_t* __restrict__ ki,
                                              uint32_t* __restrict__ order, uint32_t* __restrict__ big_list,
                                              uint32_t* __restrict__ big_count) {
  for (uint32_t e = in0 + threadIdx.x; e < in0 + (s1 - s0); e += SBT_THREADS) {
    const uint32_t j = rd[e] - d0;
    const uint32_t p = atomicAdd(&cur[j], 1u);
    Tt[p] = rt[e];
    const uint32_t v = ri[e];
    if (KK) Tk[p] = rk[e];
    else if (!LDS) Tk[p] = v;  // k_sort_big reads the global key
    Ti[p] = v;
    Ts[p] = (uint16_t)j;
  }
  slot_orders<LDS, KK, false>(Tt, Tk, Ti, Ts, s0, s1 - s0, d0, nd, cnt, kt, kk, ki, order, big_list, big_count);
}

// Block per super-bucket: its ns entries are at [in0, in0 + ns) of rd/rt/rk/ri
// and take positions [s0, s0 + ns) of order[].  In LDS when they fit (SB_CAP),
// else sorted in place in the global kt/kk/ki.
template <bool KK>
__device__ __forceinline__ void sb_sort_body(uint32_t sb, SbMap sm, uint32_t n_slots, uint32_t in0, uint32_t s0,
                                             uint32_t ns, const uint32_t* __restrict__ rd,
                                             const uint64_t* __restrict__ rt, const uint64_t* __restrict__ rk,
                                             const uint32_t* __restrict__ ri, uint64_t* __restrict__ kt,
                                             uint64_t* __restrict__ kk, uint32_t* __restrict__ ki,
                                             uint32_t* __restrict__ offsets, uint32_t* __restrict__ order,
                                             uint32_t* __restrict__ big_list, uint32_t* __restrict__ big_count,
                                             uint16_t* __restrict__ slot_spill) {
  __shared__ uint32_t cnt[SB_SLOTS_MAX + 1];
  __shared__ uint32_t cur[SB_SLOTS_MAX];
  __shared__ uint32_t wsum[SBT_THREADS / 64];
  constexpr int CAP = SB_CAP<KK>;
  __shared__ uint64_t st[CAP];
  __shared__ uint64_t sk[KK ? CAP : 1];
  __shared__ uint32_t si[CAP];
  __shared__ uint16_t ss[CAP];
  const uint32_t s1 = s0 + ns;
  const uint32_t d0 = sb * sm.spb, nd = min(sm.spb, n_slots - d0);
  const bool lds = ns <= (uint32_t)CAP;
  for (uint32_t j = threadIdx.x; j <= nd; j += SBT_THREADS) cnt[j] = 0;
  __syncthreads();
  for (uint32_t e = in0 + threadIdx.x; e < in0 + ns; e += SBT_THREADS) atomicAdd(&cnt[rd[e] - d0], 1u);
  __syncthreads();
  // exclusive scan of cnt[0..nd), nd <= SB_SLOTS_MAX
  const uint32_t tot = block_exclusive_scan<SBT_THREADS, SB_SLOTS_MAX / SBT_THREADS>(cnt, nd, wsum);
  for (uint32_t j = threadIdx.x; j < nd; j += SBT_THREADS) cur[j] = cnt[j];
  if (threadIdx.x == 0) cnt[nd] = tot;
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < nd; j += SBT_THREADS) offsets[d0 + j] = s0 + cnt[j];
  if (d0 + nd == n_slots && threadIdx.x == 0) offsets[n_slots] = s1;
  // LDS and global variants as separate inlined bodies: one generic pointer
  // would turn every access into a flat instruction waiting on both counters
  if (lds)
    sb_place_sort<true, KK>(st, sk, si, ss, in0, s0, s1, d0, nd, cnt, cur, rd, rt, rk, ri, kt, kk, ki, order,
                            big_list, big_count);
  else
    sb_place_sort<false, KK>(kt + s0, kk + s0, ki + s0, slot_spill + s0, in0, s0, s1, d0, nd, cnt, cur, rd, rt, rk,
                             ri, kt, kk, ki, order, big_list, big_count);
}

// Scan path: super-bucket sb's entries are [tile_off[sb, 0], tile_off[sb + 1, 0]).
template <bool KK>
__global__ void __launch_bounds__(SBT_THREADS)
    k_sb_sort(SbMap sm, uint32_t n_slots, const uint32_t* __restrict__ tile_off, uint32_t n_tiles,
              const uint32_t* __restrict__ rd, const uint64_t* __restrict__ rt, const uint64_t* __restrict__ rk,
              const uint32_t* __restrict__ ri, uint64_t* __restrict__ kt, uint64_t* __restrict__ kk,
              uint32_t* __restrict__ ki, uint32_t* __restrict__ offsets, uint32_t* __restrict__ order,
              uint32_t* __restrict__ big_list, uint32_t* __restrict__ big_count, uint16_t* __restrict__ slot_spill) {
  const uint32_t sb = blockIdx.x;
  const uint32_t s0 = tile_off[(size_t)sb * n_tiles], s1 = tile_off[(size_t)(sb + 1) * n_tiles];
  sb_sort_body<KK>(sb, sm, n_slots, s0, s0, s1 - s0, rd, rt, rk, ri, kt, kk, ki, offsets, order, big_list, big_count,
                   slot_spill);
}

// Output start of every super-bucket of the region path (the exclusive scan of
// its SB_SUB sub-counts), one block, for many super-buckets; with few, each
// sort block sums the counts before it itself.
__global__ void __launch_bounds__(1024) k_sb_prefix(const uint32_t* __restrict__ ctl, uint32_t n_sb,
                                                    uint32_t* __restrict__ pre) {
  __shared__ uint32_t a[SB_MAX];
  __shared__ uint32_t wsum[1024 / 64];
  for (uint32_t i = threadIdx.x; i < n_sb; i += 1024) {
    uint32_t t = 0;
#pragma unroll
    for (int k = 0; k < (int)SB_SUB; k++) t += ctl[k * SB_MAX + i];
    a[i] = t;
  }
  __syncthreads();
  block_exclusive_scan<1024, SB_MAX / 1024>(a, n_sb, wsum);
  for (uint32_t i = threadIdx.x; i < n_sb; i += 1024) pre[i] = a[i];
}

// Region path: super-bucket sb's entries are SB_SUB runs, sub-region k holding
// [sb * region + k * subcap, + count[k][sb]) (k_sb_scatter<E, true>); its output
// position is the sum of all counts of the super-buckets before it.  The block
// does nothing if a sub-region overflowed (the host then reruns the scan
// path); every block clears a share of the other parity's counters.
template <bool KK>
__global__ void __launch_bounds__(SBT_THREADS)
    k_sb_sort_region(SbMap sm, uint32_t n_slots, uint32_t n_sb, const uint32_t* __restrict__ ctl,
                     uint32_t* __restrict__ ctl_next, uint32_t region, const uint32_t* __restrict__ rd,
                     const uint64_t* __restrict__ rt, const uint64_t* __restrict__ rk,
                     const uint32_t* __restrict__ ri, uint64_t* __restrict__ kt, uint64_t* __restrict__ kk,
                     uint32_t* __restrict__ ki, uint32_t* __restrict__ offsets, uint32_t* __restrict__ order,
                     uint32_t* __restrict__ big_list, uint32_t* __restrict__ big_count,
                     uint16_t* __restrict__ slot_spill, sg_round_ret* __restrict__ ret,
                     const uint32_t* __restrict__ pre) {
  __shared__ uint32_t part[SBT_THREADS / 64];
  const uint32_t over = ctl[SB_FLAG];
  // the next parity's counters zeroed and the overflow flag published after this
  // kernel's loads: stores ahead of them made every later load wait for the stores too
  // (the flag goes to mapped host memory)
  auto epilogue = [&]() {
    for (uint32_t i = blockIdx.x * SBT_THREADS + threadIdx.x; i <= SB_FLAG; i += gridDim.x * SBT_THREADS)
      ctl_next[i] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) ret->overflow = over;
  };
  if (over) {  // uniform across the grid
    epilogue();
    return;
  }
  const uint32_t sb = blockIdx.x, subcap = region / SB_SUB;
  uint32_t s0 = 0;
  if (pre) {
    s0 = pre[sb];
  } else {
    uint32_t before = 0;
    for (uint32_t i = threadIdx.x; i < sb; i += SBT_THREADS)  // coalesced per sub-counter array
#pragma unroll
      for (int k = 0; k < (int)SB_SUB; k++) before += ctl[k * SB_MAX + i];
    for (int dd = 32; dd > 0; dd >>= 1) before += __shfl_xor(before, dd, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = before;
    __syncthreads();
    for (int w = 0; w < SBT_THREADS / 64; w++) s0 += part[w];
  }
  uint32_t sub_end[SB_SUB];  // running totals of the SB_SUB runs (wave-uniform)
  uint32_t ns = 0;
#pragma unroll
  for (int k = 0; k < (int)SB_SUB; k++) {
    ns += ctl[k * SB_MAX + sb];
    sub_end[k] = ns;
  }
  const uint32_t in0 = sb * region;  // ns <= region = SB_CAP (no overflow)
  constexpr int CAP = SB_CAP<KK>;
  constexpr int PER = (CAP + SBT_THREADS - 1) / SBT_THREADS;
  __shared__ uint32_t cnt[SB_SLOTS_MAX + 1];
  __shared__ uint32_t cur[SB_SLOTS_MAX];
  __shared__ uint32_t wsum[SBT_THREADS / 64];
  __shared__ uint64_t st[CAP];
  __shared__ uint64_t sk[KK ? CAP : 1];
  __shared__ uint32_t si[CAP];
  __shared__ uint16_t ss[pow2_ceil(CAP)];  // slot per entry, then the bitonic index array
  const uint32_t d0 = sb * sm.spb, nd = min(sm.spb, n_slots - d0);
  // the super-bucket's entries into registers: one global round trip
  uint32_t vd[PER], vi[PER];
  uint64_t vt[PER], vk[PER];
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t e = threadIdx.x + k * SBT_THREADS;
    uint32_t sub = 0, start = 0;  // entry e lies in the first run whose running total exceeds it
#pragma unroll
    for (int j = 0; j < (int)SB_SUB - 1; j++)
      if (e >= sub_end[j]) {
        sub = j + 1;
        start = sub_end[j];
      }
    // branch-free loads (a lane past the end reads the region's first slot and drops it)
    const uint32_t x = e < ns ? in0 + sub * subcap + (e - start) : in0;
    const uint32_t dd = rd[x];
    vt[k] = rt[x];
    vi[k] = ri[x];
    if (KK) vk[k] = rk[x];
    vd[k] = e < ns ? dd - d0 : NONE;
  }
  // Compressed keys (single GPU: the order key is the value, a u32): when the
  // super-bucket's arrival times span less than 2^32 ns, (t - t_min) << 32 | value
  // is unique and orders like (t, value), and the rank sort compares one word.
  bool ck = false;
  if constexpr (!KK) {
    __shared__ unsigned long long tlo[SBT_THREADS / 64], thi[SBT_THREADS / 64];
    uint64_t lo = ~0ull, hi = 0;
#pragma unroll
    for (int k = 0; k < PER; k++)
      if (vd[k] != NONE) {
        lo = min(lo, vt[k]);
        hi = max(hi, vt[k]);
      }
    for (int dd = 32; dd > 0; dd >>= 1) {
      lo = min(lo, (uint64_t)__shfl_xor((unsigned long long)lo, dd, 64));
      hi = max(hi, (uint64_t)__shfl_xor((unsigned long long)hi, dd, 64));
    }
    if ((threadIdx.x & 63) == 0) {
      tlo[threadIdx.x >> 6] = lo;
      thi[threadIdx.x >> 6] = hi;
    }
    __syncthreads();
    for (int w = 0; w < SBT_THREADS / 64; w++) {
      lo = min(lo, (uint64_t)tlo[w]);
      hi = max(hi, (uint64_t)thi[w]);
    }
    ck = ns > 0 && hi - lo < (1ull << 32);
    if (ck)
#pragma unroll
      for (int k = 0; k < PER; k++) vt[k] = ((vt[k] - lo) << 32) | vi[k];
  }
  for (uint32_t j = threadIdx.x; j <= nd; j += SBT_THREADS) cnt[j] = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; k++)
    if (vd[k] != NONE) atomicAdd(&cnt[vd[k]], 1u);
  __syncthreads();
  const uint32_t tot = block_exclusive_scan<SBT_THREADS, SB_SLOTS_MAX / SBT_THREADS>(cnt, nd, wsum);
  for (uint32_t j = threadIdx.x; j < nd; j += SBT_THREADS) cur[j] = cnt[j];
  if (threadIdx.x == 0) cnt[nd] = tot;
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < nd; j += SBT_THREADS) offsets[d0 + j] = s0 + cnt[j];
  if (d0 + nd == n_slots && threadIdx.x == 0) offsets[n_slots] = s0 + ns;
#pragma unroll
  for (int k = 0; k < PER; k++) {
    if (vd[k] == NONE) continue;
    const uint32_t p = atomicAdd(&cur[vd[k]], 1u);
    st[p] = vt[k];
    if (KK) sk[p] = vk[k];
    si[p] = vi[k];
    ss[p] = (uint16_t)vd[k];
  }
  if (ck)  // uniform per block
    slot_orders<true, KK, true, true>(st, sk, si, ss, s0, ns, d0, nd, cnt, kt, kk, ki, order, big_list, big_count);
  else
    slot_orders<true, KK, true>(st, sk, si, ss, s0, ns, d0, nd, cnt, kt, kk, ki, order, big_list, big_count);
  epilogue();
}

// Bucket sort of n entries into n_slots destination slots (see above).
// region = true tries the region path (no tile histogram, no scan); it returns
// true when it did, and the caller must then check round_ret->overflow after
// synchronising and, if set, call again with region = false (hot destinations
// that overfill a super-bucket's region; big_count zeroed again first).
template <class E>
static bool bucket_sort(sg_ctx* ctx, E src, uint32_t n, uint32_t n_slots, uint32_t* offsets, uint32_t* order,
                        uint32_t* big_count, bool region, StatsJob stats = StatsJob{}) {
  hipStream_t st = ctx->stream;
  auto stats_alone = [&] {  // the round's stats when no region scatter carries them
    if (stats.blk) hipLaunchKernelGGL(k_reduce_stats, dim3(1), dim3(1024), 0, st, stats);
    stats.blk = nullptr;
  };
  if (n_slots == 0) {
    stats_alone();
    SG_HIP(hipMemsetAsync(offsets, 0, 4, st));
    return false;
  }
  // spb slots per super-bucket: about SB_TARGET entries each, <= SB_MAX super-buckets
  if (n_slots >= (1u << 24)) throw Error(SG_ERR_INVALID_ARG, "too many destination hosts for one rank");
  uint64_t spb64 = n ? ((uint64_t)SB_TARGET<E::KK> * n_slots + n - 1) / n : SB_SLOTS_MAX;
  spb64 = std::min<uint64_t>(std::max<uint64_t>(spb64, (n_slots + SB_MAX - 1) / SB_MAX), SB_SLOTS_MAX);
  spb64 = std::max<uint64_t>(spb64, 1);
  if ((n_slots + spb64 - 1) / spb64 > (uint64_t)SB_MAX)
    throw Error(SG_ERR_INVALID_ARG, "too many destination hosts for one rank");
  SbMap sm{((1ull << 40) + spb64 - 1) / spb64, (uint32_t)spb64};
  const uint32_t n_sb = (uint32_t)((n_slots + spb64 - 1) / spb64);
  const uint32_t n_tiles = std::max<uint32_t>(1, (n + SB_TILE - 1) / SB_TILE);
  const char* env = getenv("SG_BUCKET_REGION");
  region = region && n > 0 && !(env && env[0] == '0');
  if (!region) stats_alone();
  const uint32_t reg = SB_CAP<E::KK>;  // a region is sorted in LDS in one piece
  const size_t cap = region ? std::max<size_t>((size_t)n_sb * reg, n) : n;
  uint32_t* rd = ctx->d_lists2.get<uint32_t>(cap);
  uint64_t* rt = ctx->d_keys2.get<uint64_t>(cap);
  uint64_t* rk = ctx->d_keys3.get<uint64_t>(E::KK ? cap : 1);
  uint32_t* ri = ctx->d_vals2.get<uint32_t>(cap);
  uint64_t* kt = ctx->d_keys.get<uint64_t>(n);
  uint64_t* kk = ctx->d_keys4.get<uint64_t>(n);
  uint32_t* ki = ctx->d_vals.get<uint32_t>(n);
  uint32_t* big_list = ctx->d_lists.get<uint32_t>(n_slots);
  uint16_t* spill = ctx->d_spill.get<uint16_t>(n);  // slot index per entry of super-buckets beyond SB_CAP
  if (region) {
    uint32_t* ctl = ctx->sb_ctl + (size_t)ctx->sb_parity * SB_CTL_STRIDE;
    uint32_t* ctl_next = ctx->sb_ctl + (size_t)(ctx->sb_parity ^ 1) * SB_CTL_STRIDE;
    ctx->sb_parity ^= 1;
    // Two levels when a tile would spread over so many super-buckets that its
    // runs are a few entries long (C5: 10M entries, 3,847 super-buckets, about
    // one entry per super-bucket per tile -- every store scattered, one global
    // atomic per entry).  The first level scatters into at most 256 coarse
    // buckets of cpb consecutive super-buckets (runs of 16+ entries), the second
    // level scatters each coarse bucket's tiles into its cpb super-buckets.
    const char* tl_env = getenv("SG_BUCKET_TWO_LEVEL");  // 0 never, 1 always (tests), else when runs are short
    const int two_env = tl_env && *tl_env ? atoi(tl_env) : -1;
    const bool two = two_env == 1 || (two_env != 0 && n_sb > 512);
    if (two) {
      const uint32_t cpb = std::max<uint32_t>(2, (n_sb + CB_MAX - 1) / CB_MAX), n_cb = (n_sb + cpb - 1) / cpb;
      static_assert(SB_MAX / CB_MAX <= CB_MAX, "a coarse bucket's super-buckets must fit CB_MAX");
      SbMap cm{((1ull << 40) + (uint64_t)spb64 * cpb - 1) / ((uint64_t)spb64 * cpb), (uint32_t)(spb64 * cpb)};
      // per (coarse bucket, XCD) sub-region: 1.25x its mean share + 1024, in whole tiles
      const uint64_t mean = ((uint64_t)n + (uint64_t)n_cb * SB_SUB - 1) / ((uint64_t)n_cb * SB_SUB);
      const uint64_t subcap = (mean + mean / 4 + 1024 + SB_TILE - 1) / SB_TILE * SB_TILE;
      const uint64_t creg = subcap * SB_SUB, ctot = creg * n_cb;
      if (ctot >= (1ull << 31)) throw Error(SG_ERR_INVALID_ARG, "round too large for the bucketing workspace");
      uint32_t* cctl = ctx->sb_ctl + (size_t)(2 + ctx->sb_parity_c) * SB_CTL_STRIDE;
      uint32_t* cctl_next = ctx->sb_ctl + (size_t)(2 + (ctx->sb_parity_c ^ 1)) * SB_CTL_STRIDE;
      ctx->sb_parity_c ^= 1;
      uint32_t* cd = ctx->d_cd.get<uint32_t>(ctot);
      uint64_t* ct = ctx->d_ct.get<uint64_t>(ctot);
      uint64_t* ck = ctx->d_ck.get<uint64_t>(E::KK ? ctot : 1);
      uint32_t* ci = ctx->d_ci.get<uint32_t>(ctot);
      {
        TimedLaunch tl(ctx, "scatter", 32.0 * n);
        hipLaunchKernelGGL((k_sb_scatter<E, true, CB_MAX>), dim3(n_tiles + (stats.blk ? 1 : 0)), dim3(SBS_THREADS), 0, st,
                           src, n, cm, n_cb, nullptr, cctl, (uint32_t)creg, cd, ct, ck, ci, stats);
      }
      CoarseEntries<E::KK> ce{cd, ct, ck, ci, cctl, cctl_next, (uint32_t)creg, (uint32_t)subcap, cpb};
      {
        TimedLaunch tl(ctx, "scatter2", 32.0 * n);
        hipLaunchKernelGGL((k_sb_scatter<CoarseEntries<E::KK>, true, CB_MAX>), dim3((uint32_t)(ctot / SB_TILE)),
                           dim3(SBS_THREADS), 0, st, ce, (uint32_t)ctot, sm, n_sb, nullptr, ctl, reg, rd, rt, rk, ri,
                           StatsJob{});
      }
    } else {
      TimedLaunch tl(ctx, "scatter", 32.0 * n);
      hipLaunchKernelGGL((k_sb_scatter<E, true>), dim3(n_tiles + (stats.blk ? 1 : 0)), dim3(SBS_THREADS), 0, st, src,
                         n, sm, n_sb, nullptr, ctl, reg, rd, rt, rk, ri, stats);
    }
    // many super-buckets: their output starts from one scan, not a sum per sort block
    uint32_t* pre = n_sb > 512 ? ctx->d_cur.get<uint32_t>(n_sb) : nullptr;
    if (pre) hipLaunchKernelGGL(k_sb_prefix, dim3(1), dim3(1024), 0, st, ctl, n_sb, pre);
    {
      TimedLaunch tl(ctx, "sort_small", 24.0 * n + 4.0 * n_slots);
      hipLaunchKernelGGL(k_sb_sort_region<E::KK>, dim3(n_sb), dim3(SBT_THREADS), 0, st, sm, n_slots, n_sb, ctl,
                         ctl_next, reg, rd, rt, rk, ri, kt, kk, ki, offsets, order, big_list, big_count, spill,
                         ctx->round_ret, (const uint32_t*)pre);
    }
  } else {
    const size_t nh = (size_t)n_sb * n_tiles;
    uint32_t* hist = ctx->d_cnt.get<uint32_t>(nh + 1);
    uint32_t* toff = ctx->d_scan.get<uint32_t>(nh + 1);
    {
      TimedLaunch tl(ctx, "scatter", 56.0 * n);
      if (n) hipLaunchKernelGGL(k_sb_hist<E>, dim3(n_tiles), dim3(SB_THREADS), 0, st, src, n, sm, n_sb, hist);
      else SG_HIP(hipMemsetAsync(hist, 0, nh * 4, st));
      exclusive_scan_u32(ctx, hist, toff, (uint32_t)nh);
      if (n)
        hipLaunchKernelGGL((k_sb_scatter<E, false>), dim3(n_tiles), dim3(SBS_THREADS), 0, st, src, n, sm, n_sb, toff,
                           nullptr, 0u, rd, rt, rk, ri, StatsJob{});
    }
    {
      TimedLaunch tl(ctx, "sort_small", 48.0 * n + 4.0 * n_slots);
      hipLaunchKernelGGL(k_sb_sort<E::KK>, dim3(n_sb), dim3(SBT_THREADS), 0, st, sm, n_slots, toff, n_tiles, rd, rt,
                         rk, ri, kt, kk, ki, offsets, order, big_list, big_count, spill);
    }
  }
  if (region) {  // big slots were sorted in-block
    SG_CHECK_LAUNCH();
    return true;
  }
  uint64_t* kt2 = ctx->d_keys2.get<uint64_t>(n);  // rd/rt are free again
  uint64_t* kk2 = ctx->d_keys3.get<uint64_t>(n);
  uint32_t* ki2 = ctx->d_vals2.get<uint32_t>(n);
  {
    TimedLaunch tl(ctx, "sort_big", 0.0);
    hipLaunchKernelGGL(k_sort_big, dim3(std::min<uint32_t>(std::max(n_slots, 1u), 2048)), dim3(SORT_BLOCK), 0, st,
                       offsets, big_list, big_count, kt, kk, ki, kt2, kk2, ki2, order);
  }
  SG_CHECK_LAUNCH();
  return region;
}

struct RoundWork {
  uint32_t *host_off, *big_count, *dst_host;
  uint64_t* ctr_start;
  bool walked;     // the walk ran and its stats reach round_ret (P > 0)
  StatsJob stats;  // set when the caller launches the stats reduction (fused)
};

// Shared source half of a round: host offsets + walk.  Leaves per-packet
// dst_host (NONE unless delivered) and the round stats.
static RoundWork source_phase(sg_ctx* ctx, sg_hosts* hs, const sg_table* tab, const sg_round* rd,
                              const sg_packets* pk, uint8_t* status, uint64_t* deliver, uint64_t* eid,
                              bool want_ctr_start, bool fuse_stats = false, unsigned long long* stats_row = nullptr) {
  hipStream_t st = ctx->stream;
  const uint32_t P = pk->n_packets, H = hs->n;
  RoundWork w;
  // workspace: [host_off H+1][big_count 1]; k_host_off writes every host_off
  // entry of well-grouped packets (else it flags an error and the walk skips),
  // k_reduce_stats zeroes big_count: no fills on the round's path
  uint32_t* ws = ctx->d_seg.get<uint32_t>((size_t)H + 8);
  w.host_off = ws;
  w.big_count = ws + (size_t)H + 1;
  w.dst_host = ctx->d_dst.get<uint32_t>(P);
  w.ctr_start = want_ctr_start ? ctx->d_ctr0.get<uint64_t>(H) : nullptr;
  w.walked = P > 0;
  w.stats = StatsJob{};
  if (w.ctr_start) SG_HIP(hipMemcpyAsync(w.ctr_start, hs->ctr, (size_t)H * 8, hipMemcpyDeviceToDevice, st));
  if (!P) {
    SG_HIP(hipMemsetAsync(w.big_count, 0, 4, st));
    if (stats_row) {  // no packets: delivered 0, no minima, no source-phase errors
      ctx->round_ret->err = 0;  // (mapped; the previous round's writes were synchronised)
      const unsigned long long none[3] = {0, ~0ull, ~0ull};
      SG_HIP(hipMemcpyAsync(stats_row, none, sizeof(none), hipMemcpyHostToDevice, st));
      SG_HIP(hipStreamSynchronize(st));  // (the host array leaves scope; an empty round only)
    }
    return w;
  }
  {
    TimedLaunch tl(ctx, "seg_bounds", 4.0 * P + 4.0 * H);
    // the sending hosts' route rows are checked against the shard only when some host's
    // row lies outside it: a whole table, or a shard holding every host's row, needs no
    // route gather on the round's path (C4: k_host_off4 7.7 -> 6.1 us, r04y)
    const bool all_in = H && hs->min_route >= tab->row_begin && hs->max_route - tab->row_begin < tab->n_rows;
    const uint32_t* route_chk = all_in ? nullptr : hs->route;
    if (((uintptr_t)pk->src_host & 15) == 0 && P < (1u << 30))  // one thread per 4 packets, no grid stride
      hipLaunchKernelGGL(k_host_off4, dim3((unsigned)(((size_t)P + 4) / 4 + 255) / 256), dim3(256), 0, st,
                         pk->src_host, P, H, w.host_off, ctx->round_err, route_chk, tab->row_begin, tab->n_rows);
    else
      hipLaunchKernelGGL(k_host_off, dim3(grid_for((size_t)P + 1, 256, 1u << 20)), dim3(256), 0, st, pk->src_host, P,
                         H, w.host_off, ctx->round_err, route_chk, tab->row_begin, tab->n_rows);
  }
  WalkArgs a;
  a.src = pk->src_host;
  a.dst_ip = pk->dst_ipv4;
  a.payload = pk->payload_len;
  a.send = pk->send_time_ns;
  a.skip = pk->rng_skip;
  a.P = P;
  a.H = H;
  a.host_off = w.host_off;
  a.route = hs->route;
  a.rng = hs->rng;
  a.ctr = hs->ctr;
  a.map = HostMap{hs->ip_base, hs->dense_span, hs->n, hs->dense, hs->sorted_ip, hs->sorted_host};
  a.tab_lat = tab->latency_ns;
  a.tab_loss = tab->packet_loss;
  a.tab_key = tab->path_key;
  a.n_cols = tab->n_cols;
  a.row_begin = tab->row_begin;
  a.n_rows = tab->n_rows;
  a.round_end = rd->round_end_ns;
  a.sim_end = rd->sim_end_ns;
  a.bootstrap_end = rd->bootstrap_end_ns;
  a.status = status;
  a.deliver = deliver;
  a.eid = eid;
  a.dst_host = w.dst_host;
  const uint32_t walk_blocks = (H + WALK_HOSTS - 1) / WALK_HOSTS;
  a.blk_stats = ctx->d_blk.get<unsigned long long>(3 * (size_t)walk_blocks);
  a.err = ctx->round_err;
  a.pair_count = ctx->pair_count;
  if (a.pair_count && ctx->pair_count_cells < (uint64_t)tab->n_rows * tab->n_cols)
    throw Error(SG_ERR_INVALID_ARG, "packet counters smaller than the routing table");
  {
    // per packet: 20 B in, 12 B (8 B packed) path gather, 4 B dst map, 21 B out (status, time, id),
    // 4 B dst scratch; per host: 8 B segment, 4 B route, 32+32 B RNG, 8+8 B event counter
    TimedLaunch tl(ctx, "walk", (tab->path_key ? 57.0 : 61.0) * P + 92.0 * H);
    auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(walk_blocks), dim3(WALK_THREADS), 0, st, a); };
    if (a.pair_count) {
      if (a.tab_key && a.skip) go(k_walk<true, true, true>);
      else if (a.tab_key) go(k_walk<true, false, true>);
      else if (a.skip) go(k_walk<false, true, true>);
      else go(k_walk<false, false, true>);
    } else if (a.tab_key && a.skip) {
      go(k_walk<true, true>);
    } else if (a.tab_key) {
      go(k_walk<true, false>);
    } else if (a.skip) {
      go(k_walk<false, true>);
    } else {
      go(k_walk<false, false>);
    }
  }
  const StatsJob sj{a.blk_stats, walk_blocks, ctx->round_err, w.big_count, ctx->round_ret, stats_row};
  if (fuse_stats)
    w.stats = sj;
  else
    hipLaunchKernelGGL(k_reduce_stats, dim3(1), dim3(1024), 0, st, sj);
  SG_CHECK_LAUNCH();
  return w;
}

static void finish(sg_ctx* ctx, const RoundWork& w, sg_round_stats* stats) {
  SG_HIP(hipStreamSynchronize(ctx->stream));
  unsigned long long s[3] = {0, ~0ull, ~0ull};
  uint32_t err = 0;
  if (w.walked) {  // written by k_reduce_stats into mapped host memory; the sync made it visible
    const volatile sg_round_ret* r = ctx->round_ret;
    for (int i = 0; i < 3; i++) s[i] = r->stats[i];
    err = r->err;
  }
  fail_flags(err);
  if (stats) {
    stats->n_delivered = s[0];
    stats->min_deliver_time_ns = s[1];
    stats->min_used_latency_ns = s[2];
  }
}

static void deliver_round(sg_ctx* ctx, sg_hosts* hs, const sg_table* tab, const sg_round* rd,
                          const sg_packets* pk, sg_deliveries* out, sg_round_stats* stats) {
  const uint32_t P = pk->n_packets, H = hs->n;
  RoundWork w = source_phase(ctx, hs, tab, rd, pk, out->status, out->deliver_time_ns, out->event_id, false, true);
  const PacketEntries E{w.dst_host, out->deliver_time_ns};
  const bool region = bucket_sort(ctx, E, P, H, out->dst_offsets, out->dst_order, w.big_count, true, w.stats);
  finish(ctx, w, stats);
  if (region && ctx->round_ret->overflow) {  // a hot destination overfilled its region
    SG_HIP(hipMemsetAsync(w.big_count, 0, 4, ctx->stream));
    bucket_sort(ctx, E, P, H, out->dst_offsets, out->dst_order, w.big_count, false);
    SG_HIP(hipStreamSynchronize(ctx->stream));
  }
}

static void deliver_source(sg_ctx* ctx, sg_hosts* hs, const sg_table* tab, const sg_round* rd,
                           const sg_packets* pk, uint8_t* status, uint64_t* deliver, uint64_t* eid,
                           const uint32_t* owner, uint32_t n_ranks, sg_record* send, uint32_t* send_counts,
                           sg_round_stats* stats) {
  hipStream_t st = ctx->stream;
  const uint32_t P = pk->n_packets;
  RoundWork w = source_phase(ctx, hs, tab, rd, pk, status, deliver, eid, true);
  const uint32_t nb = std::max<uint32_t>(1, std::min<uint32_t>(grid_for(P, PACK_BLOCK * 8), 2048));
  uint32_t* bc = ctx->d_cnt.get<uint32_t>((size_t)n_ranks * nb + 1);
  uint32_t* bo = ctx->d_scan.get<uint32_t>((size_t)n_ranks * nb + 1);
  SG_HIP(hipMemsetAsync(bc, 0, ((size_t)n_ranks * nb + 1) * 4, st));
  if (P) {
    TimedLaunch tl(ctx, "pack", 4.0 * P + 32.0 * P);
    hipLaunchKernelGGL(k_owner_count, dim3(nb), dim3(PACK_BLOCK), 0, st, w.dst_host, P, owner, n_ranks, bc);
  }
  exclusive_scan_u32(ctx, bc, bo, n_ranks * nb);
  if (P) {
    hipLaunchKernelGGL(k_owner_scatter, dim3(nb), dim3(PACK_BLOCK), 0, st, pk->src_host, w.dst_host, deliver, eid,
                       w.ctr_start, P, owner, n_ranks, bo, send, (sg_record*)nullptr, 0u);
    SG_CHECK_LAUNCH();
  }
  std::vector<uint32_t> starts((size_t)n_ranks * nb + 1);
  SG_HIP(hipMemcpyAsync(starts.data(), bo, starts.size() * 4, hipMemcpyDeviceToHost, st));
  finish(ctx, w, stats);  // synchronises the stream
  for (uint32_t r = 0; r < n_ranks; r++) send_counts[r] = starts[(size_t)(r + 1) * nb] - starts[(size_t)r * nb];
}

// The fixed-split exchange's source half: as deliver_source, but nothing is read
// back -- the records for rank r go to padded[r * cap + k] (k < cap; the rest to
// their compact positions in `send`), and xrow (device) receives the round's
// stats and the per-rank counts for the caller's all-gather.
static void deliver_source_padded(sg_ctx* ctx, sg_hosts* hs, const sg_table* tab, const sg_round* rd,
                                  const sg_packets* pk, uint8_t* status, uint64_t* deliver, uint64_t* eid,
                                  const uint32_t* owner, uint32_t n_ranks, uint32_t cap, sg_record* padded,
                                  sg_record* send, unsigned long long* xrow) {
  hipStream_t st = ctx->stream;
  const uint32_t P = pk->n_packets;
  RoundWork w = source_phase(ctx, hs, tab, rd, pk, status, deliver, eid, true, false, xrow);
  const uint32_t nb = std::max<uint32_t>(1, std::min<uint32_t>(grid_for(P, PACK_BLOCK * 8), 2048));
  uint32_t* bc = ctx->d_cnt.get<uint32_t>((size_t)n_ranks * nb + 1);
  uint32_t* bo = ctx->d_scan.get<uint32_t>((size_t)n_ranks * nb + 1);
  SG_HIP(hipMemsetAsync(bc, 0, ((size_t)n_ranks * nb + 1) * 4, st));
  if (P) {
    TimedLaunch tl(ctx, "pack", 4.0 * P + 32.0 * P);
    hipLaunchKernelGGL(k_owner_count, dim3(nb), dim3(PACK_BLOCK), 0, st, w.dst_host, P, owner, n_ranks, bc);
  }
  exclusive_scan_u32(ctx, bc, bo, n_ranks * nb);
  if (P)
    hipLaunchKernelGGL(k_owner_scatter, dim3(nb), dim3(PACK_BLOCK), 0, st, pk->src_host, w.dst_host, deliver, eid,
                       w.ctr_start, P, owner, n_ranks, bo, send, padded, cap);
  hipLaunchKernelGGL(k_xrow_counts, dim3(1), dim3(MAX_RANKS), 0, st, bo, nb, n_ranks, xrow);
  SG_CHECK_LAUNCH();
}

// The destination half of a fixed-split exchange: recv holds n_ranks blocks of
// cap records (block b from rank b), xall the all-gathered rows.  One
// synchronisation: then the source phase's and the bucketing's errors, the
// global stats, this rank's receive counts and the largest pair count are read
// from the mapped return block.
static void deliver_bucket_padded(sg_ctx* ctx, const sg_record* recv, uint32_t n_ranks, uint32_t cap,
                                  const unsigned long long* xall, uint32_t rank, const uint32_t* local, uint32_t H,
                                  uint32_t n_local, uint32_t* order, uint32_t* offsets, sg_round_stats* stats,
                                  uint32_t* recv_counts, uint32_t* pair_max) {
  hipStream_t st = ctx->stream;
  uint32_t* ws = ctx->d_seg.get<uint32_t>(8);
  uint32_t* big_count = ws;
  uint32_t* err = ws + 1;
  SG_HIP(hipMemsetAsync(ws, 0, 8 * 4, st));
  const uint64_t n64 = (uint64_t)n_ranks * cap;
  if (n64 >= (1ull << 31)) throw Error(SG_ERR_INVALID_ARG, "padded exchange too large (n_ranks x cap >= 2^31)");
  const PaddedRecordEntries E{recv, local, H, err, cap, 3 + n_ranks, rank, xall};
  const bool region = bucket_sort(ctx, E, (uint32_t)n64, n_local, offsets, order, big_count, true);
  hipLaunchKernelGGL(k_xall_reduce, dim3(1), dim3(MAX_RANKS), 0, st, xall, n_ranks, rank, err, ctx->round_ret);
  SG_CHECK_LAUNCH();
  SG_HIP(hipStreamSynchronize(st));
  const volatile sg_round_ret* r = ctx->round_ret;
  fail_flags(r->err);
  if (region && r->overflow) {  // a hot destination overfilled its region
    SG_HIP(hipMemsetAsync(ws, 0, 8 * 4, st));
    bucket_sort(ctx, E, (uint32_t)n64, n_local, offsets, order, big_count, false);
    uint32_t h_err = 0;
    copy_to_host(ctx, &h_err, err, 4);
    fail_flags(h_err);
  }
  if (stats) {
    stats->n_delivered = r->stats[0];
    stats->min_deliver_time_ns = r->stats[1];
    stats->min_used_latency_ns = r->stats[2];
  }
  if (recv_counts)
    for (uint32_t b = 0; b < n_ranks; b++) recv_counts[b] = r->recv_cnt[b];
  if (pair_max) *pair_max = r->pair_max;
}

static void deliver_bucket(sg_ctx* ctx, const sg_record* recv, uint32_t n, const uint32_t* local, uint32_t H,
                           uint32_t n_local, uint32_t* order, uint32_t* offsets) {
  hipStream_t st = ctx->stream;
  uint32_t* ws = ctx->d_seg.get<uint32_t>(8);
  uint32_t* big_count = ws;
  uint32_t* err = ws + 1;
  SG_HIP(hipMemsetAsync(ws, 0, 8 * 4, st));
  const RecordEntries E{recv, local, H, err};
  const bool region = bucket_sort(ctx, E, n, n_local, offsets, order, big_count, true);
  uint32_t h_err = 0;
  copy_to_host(ctx, &h_err, err, 4);
  fail_flags(h_err);
  if (region && ctx->round_ret->overflow) {  // a hot destination overfilled its region
    SG_HIP(hipMemsetAsync(ws, 0, 8 * 4, st));
    bucket_sort(ctx, E, n, n_local, offsets, order, big_count, false);
    copy_to_host(ctx, &h_err, err, 4);
    fail_flags(h_err);
  }
}

void launch_group_offsets(sg_ctx* ctx, const uint32_t* key, uint32_t n, uint32_t n_groups, uint32_t* off,
                          uint32_t* err) {
  hipLaunchKernelGGL(k_host_off, dim3(grid_for((size_t)n + 1, 256, 16384)), dim3(256), 0, ctx->stream, key, n,
                     n_groups, off, err);
  SG_CHECK_LAUNCH();
}

// sg_hosts_skip: host ids[i] (unique) advances its stream by steps[i] next_u64 steps.
__global__ void __launch_bounds__(256) k_hosts_skip(const uint32_t* __restrict__ ids, const uint64_t* __restrict__ steps,
                                                    uint32_t m, uint32_t H, uint64_t* __restrict__ rng) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= m) return;
  const size_t h = ids[i];
  Xoshiro x{rng[h], rng[(size_t)H + h], rng[2 * (size_t)H + h], rng[3 * (size_t)H + h]};
  for (uint64_t z = steps[i]; z; z--) (void)x.next_u64();
  rng[h] = x.s0;
  rng[(size_t)H + h] = x.s1;
  rng[2 * (size_t)H + h] = x.s2;
  rng[3 * (size_t)H + h] = x.s3;
}

// Path-key table: (lat << 32) | bits(loss) per cell, so the walk's path gather
// is one 8-byte word.  Streaming, coalesced: 12 B in + 8 B out per cell.
__global__ void __launch_bounds__(256) k_table_pack(const uint64_t* __restrict__ lat, const float* __restrict__ loss,
                                                    size_t cells, uint64_t* __restrict__ key, uint32_t* wide) {
  bool over = false;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < cells; i += (size_t)gridDim.x * 256) {
    const uint64_t l = lat[i];
    over |= (l >> 32) != 0;
    key[i] = (l << 32) | __float_as_uint(loss[i]);
  }
  if (__any(over) && (threadIdx.x & 63) == 0) *wide = 1;  // rare: one store per wave that saw one
}

static void table_pack(sg_ctx* ctx, const sg_table* tab, size_t cells, uint64_t* key, uint32_t* packable) {
  hipStream_t st = ctx->stream;
  uint32_t* wide = ctx->d_seg.get<uint32_t>(1);
  SG_HIP(hipMemsetAsync(wide, 0, 4, st));
  if (cells) {
    TimedLaunch tl(ctx, "table_pack", 20.0 * cells);
    hipLaunchKernelGGL(k_table_pack, dim3(grid_for(cells, 256, 8192)), dim3(256), 0, st, tab->latency_ns,
                       tab->packet_loss, cells, key, wide);
    SG_CHECK_LAUNCH();
  }
  uint32_t h = 0;
  copy_to_host(ctx, &h, wide, 4);
  *packable = h ? 0 : 1;
}

}  // namespace sg

extern "C" {

int32_t sg_hosts_create(sg_ctx* ctx, uint32_t n_hosts, const uint32_t* host_ipv4,
                        const uint32_t* host_route_idx, const uint64_t* host_seed,
                        sg_hosts** out) {
  if (!out) return SG_ERR_INVALID_ARG;
  *out = nullptr;
  sg_hosts* hs = nullptr;
  int32_t rc = sg::guarded(ctx, [&] {
    using namespace sg;
    if (n_hosts && (!host_ipv4 || !host_route_idx || !host_seed))
      throw Error(SG_ERR_INVALID_ARG, "null host array");
    hs = new sg_hosts();
    hs->ctx = ctx;
    hs->n = n_hosts;
    hipStream_t st = ctx->stream;
    const size_t n = n_hosts;
    SG_HIP(hipMalloc(&hs->route, std::max<size_t>(n * 4, 16)));
    SG_HIP(hipMalloc(&hs->rng, std::max<size_t>(n * 32, 16)));
    SG_HIP(hipMalloc(&hs->ctr, std::max<size_t>(n * 8, 16)));
    uint64_t* d_seed = nullptr;
    SG_HIP(hipMalloc(&d_seed, std::max<size_t>(n * 8, 16)));
    hs->min_route = n_hosts ? ~0u : 0u;
    for (uint32_t h = 0; h < n_hosts; h++) {
      hs->max_route = std::max(hs->max_route, host_route_idx[h]);
      hs->min_route = std::min(hs->min_route, host_route_idx[h]);
    }
    std::vector<std::pair<uint32_t, uint32_t>> ips(n);
    for (uint32_t h = 0; h < n_hosts; h++) ips[h] = {host_ipv4[h], h};
    std::sort(ips.begin(), ips.end());
    for (size_t k = 1; k < n; k++)
      if (ips[k].first == ips[k - 1].first) {
        (void)hipFree(d_seed);
        throw Error(SG_ERR_DUPLICATE_IP, "IP address has already been assigned");
      }
    if (n) {
      SG_HIP(hipMemcpyAsync(hs->route, host_route_idx, n * 4, hipMemcpyHostToDevice, st));
      SG_HIP(hipMemcpyAsync(d_seed, host_seed, n * 8, hipMemcpyHostToDevice, st));
      SG_HIP(hipMemsetAsync(hs->ctr, 0, n * 8, st));
      hipLaunchKernelGGL(k_seed_hosts, dim3(grid_for(n, 256)), dim3(256), 0, st, d_seed, n_hosts, hs->rng);
      SG_CHECK_LAUNCH();
      uint64_t span = (uint64_t)ips.back().first - ips.front().first + 1;
      if (span <= 4 * (uint64_t)n + 4096) {
        hs->ip_base = ips.front().first;
        hs->dense_span = (uint32_t)span;
        std::vector<uint2> dense(span, make_uint2(NONE, 0));
        for (auto& p : ips) dense[p.first - hs->ip_base] = make_uint2(p.second, host_route_idx[p.second]);
        SG_HIP(hipMalloc(&hs->dense, span * 8));
        SG_HIP(hipMemcpyAsync(hs->dense, dense.data(), span * 8, hipMemcpyHostToDevice, st));
        SG_HIP(hipStreamSynchronize(st));
      } else {
        std::vector<uint32_t> a(n);
        std::vector<uint2> b(n);
        for (size_t k = 0; k < n; k++) {
          a[k] = ips[k].first;
          b[k] = make_uint2(ips[k].second, host_route_idx[ips[k].second]);
        }
        SG_HIP(hipMalloc(&hs->sorted_ip, n * 4));
        SG_HIP(hipMalloc(&hs->sorted_host, n * 8));
        SG_HIP(hipMemcpyAsync(hs->sorted_ip, a.data(), n * 4, hipMemcpyHostToDevice, st));
        SG_HIP(hipMemcpyAsync(hs->sorted_host, b.data(), n * 8, hipMemcpyHostToDevice, st));
        SG_HIP(hipStreamSynchronize(st));
      }
    }
    SG_HIP(hipStreamSynchronize(st));
    (void)hipFree(d_seed);
  });
  if (rc != SG_OK) {
    delete hs;
    return rc;
  }
  *out = hs;
  return SG_OK;
}

int32_t sg_hosts_get_state(sg_hosts* hs, uint64_t* rng_state, uint64_t* event_ctr) {
  if (!hs) return SG_ERR_INVALID_ARG;
  return sg::guarded(hs->ctx, [&] {
    const size_t n = hs->n;
    if (!n) return;
    std::vector<uint64_t> soa(4 * n);
    SG_HIP(hipMemcpyAsync(soa.data(), hs->rng, n * 32, hipMemcpyDeviceToHost, hs->ctx->stream));
    if (event_ctr)
      SG_HIP(hipMemcpyAsync(event_ctr, hs->ctr, n * 8, hipMemcpyDeviceToHost, hs->ctx->stream));
    SG_HIP(hipStreamSynchronize(hs->ctx->stream));
    if (rng_state)
      for (size_t h = 0; h < n; h++)
        for (int k = 0; k < 4; k++) rng_state[4 * h + k] = soa[k * n + h];
  });
}

int32_t sg_hosts_set_state(sg_hosts* hs, const uint64_t* rng_state, const uint64_t* event_ctr) {
  if (!hs) return SG_ERR_INVALID_ARG;
  return sg::guarded(hs->ctx, [&] {
    const size_t n = hs->n;
    if (!n) return;
    if (rng_state) {
      std::vector<uint64_t> soa(4 * n);
      for (size_t h = 0; h < n; h++)
        for (int k = 0; k < 4; k++) soa[k * n + h] = rng_state[4 * h + k];
      SG_HIP(hipMemcpyAsync(hs->rng, soa.data(), n * 32, hipMemcpyHostToDevice, hs->ctx->stream));
      SG_HIP(hipStreamSynchronize(hs->ctx->stream));
    }
    if (event_ctr) {
      SG_HIP(hipMemcpyAsync(hs->ctr, event_ctr, n * 8, hipMemcpyHostToDevice, hs->ctx->stream));
      SG_HIP(hipStreamSynchronize(hs->ctx->stream));
    }
  });
}

int32_t sg_hosts_skip(sg_hosts* hs, uint32_t n, const uint32_t* host_ids, const uint64_t* steps) {
  if (!hs || (n && (!host_ids || !steps))) return SG_ERR_INVALID_ARG;
  return sg::guarded(hs->ctx, [&] {
    // one entry per host (a host may repeat in the call), then one device thread per host
    std::vector<std::pair<uint32_t, uint64_t>> hv(n);
    for (uint32_t i = 0; i < n; i++) {
      if (host_ids[i] >= hs->n) throw sg::Error(SG_ERR_INVALID_ARG, "sg_hosts_skip: host out of range");
      hv[i] = {host_ids[i], steps[i]};
    }
    std::sort(hv.begin(), hv.end());
    std::vector<uint32_t> ids;
    std::vector<uint64_t> tot;
    for (auto& e : hv) {
      if (!ids.empty() && ids.back() == e.first) {
        tot.back() += e.second;
      } else {
        ids.push_back(e.first);
        tot.push_back(e.second);
      }
    }
    if (ids.empty()) return;
    const uint32_t m = (uint32_t)ids.size();
    uint32_t* d_ids = hs->ctx->d_lists.get<uint32_t>(m);
    uint64_t* d_tot = hs->ctx->d_keys.get<uint64_t>(m);
    hipStream_t st = hs->ctx->stream;
    SG_HIP(hipMemcpyAsync(d_ids, ids.data(), (size_t)m * 4, hipMemcpyHostToDevice, st));
    SG_HIP(hipMemcpyAsync(d_tot, tot.data(), (size_t)m * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(sg::k_hosts_skip, dim3(sg::grid_for(m, 256)), dim3(256), 0, st, d_ids, d_tot, m, hs->n, hs->rng);
    SG_CHECK_LAUNCH();
    SG_HIP(hipStreamSynchronize(st));
  });
}

void sg_hosts_destroy(sg_hosts* hs) {
  if (!hs) return;
  if (hs->ctx) (void)hipSetDevice(hs->ctx->device);
  delete hs;
}

int32_t sg_deliver_round(sg_ctx* ctx, sg_hosts* hosts, const sg_table* table, const sg_round* round,
                         const sg_packets* packets, sg_deliveries* out, sg_round_stats* stats) {
  return sg::guarded(ctx, [&] {
    using namespace sg;
    if (!hosts || hosts->ctx != ctx || !table || !round || !packets || !out)
      throw Error(SG_ERR_INVALID_ARG, "null argument");
    if (!out->dst_offsets) throw Error(SG_ERR_INVALID_ARG, "null dst_offsets");
    if (hosts->n && hosts->max_route >= table->n_cols)
      throw Error(SG_ERR_INVALID_ARG, "a host's routing index is outside the table's columns");
    if (packets->n_packets &&
        (!packets->src_host || !packets->dst_ipv4 || !packets->payload_len || !packets->send_time_ns ||
         !out->status || !out->deliver_time_ns || !out->event_id || !out->dst_order ||
         (!table->path_key && (!table->latency_ns || !table->packet_loss))))
      throw Error(SG_ERR_INVALID_ARG, "null packet or output array");
    deliver_round(ctx, hosts, table, round, packets, out, stats);
  });
}

int32_t sg_ctx_set_packet_counters(sg_ctx* ctx, uint64_t* counts, uint64_t n_cells) {
  if (!ctx || (counts && !n_cells)) return SG_ERR_INVALID_ARG;
  ctx->pair_count = (unsigned long long*)counts;
  ctx->pair_count_cells = counts ? n_cells : 0;
  return SG_OK;
}

}  // extern "C"

extern "C" {

int32_t sg_deliver_source(sg_ctx* ctx, sg_hosts* hosts, const sg_table* table, const sg_round* round,
                          const sg_packets* packets, uint8_t* status, uint64_t* deliver_time_ns,
                          uint64_t* event_id, const uint32_t* host_owner, uint32_t n_ranks, sg_record* send,
                          uint32_t* send_counts, sg_round_stats* stats) {
  return sg::guarded(ctx, [&] {
    using namespace sg;
    if (!hosts || hosts->ctx != ctx || !table || !round || !packets || !host_owner || !send_counts)
      throw Error(SG_ERR_INVALID_ARG, "null argument");
    if (n_ranks == 0 || n_ranks > MAX_RANKS) throw Error(SG_ERR_INVALID_ARG, "n_ranks must be in [1, 64]");
    if (hosts->n && hosts->max_route >= table->n_cols)
      throw Error(SG_ERR_INVALID_ARG, "a host's routing index is outside the table's columns");
    if (packets->n_packets &&
        (!packets->src_host || !packets->dst_ipv4 || !packets->payload_len || !packets->send_time_ns || !status ||
         !deliver_time_ns || !event_id || !send || (!table->path_key && (!table->latency_ns || !table->packet_loss))))
      throw Error(SG_ERR_INVALID_ARG, "null packet or output array");
    deliver_source(ctx, hosts, table, round, packets, status, deliver_time_ns, event_id, host_owner, n_ranks, send,
                   send_counts, stats);
  });
}

int32_t sg_deliver_source_padded(sg_ctx* ctx, sg_hosts* hosts, const sg_table* table, const sg_round* round,
                                 const sg_packets* packets, uint8_t* status, uint64_t* deliver_time_ns,
                                 uint64_t* event_id, const uint32_t* host_owner, uint32_t n_ranks, uint32_t cap,
                                 sg_record* send_padded, sg_record* send, uint64_t* xrow) {
  return sg::guarded(ctx, [&] {
    using namespace sg;
    if (!hosts || hosts->ctx != ctx || !table || !round || !packets || !host_owner || !send_padded || !xrow)
      throw Error(SG_ERR_INVALID_ARG, "null argument");
    if (n_ranks == 0 || n_ranks > MAX_RANKS) throw Error(SG_ERR_INVALID_ARG, "n_ranks must be in [1, 64]");
    if (cap == 0) throw Error(SG_ERR_INVALID_ARG, "cap must be positive");
    if (hosts->n && hosts->max_route >= table->n_cols)
      throw Error(SG_ERR_INVALID_ARG, "a host's routing index is outside the table's columns");
    if (packets->n_packets &&
        (!packets->src_host || !packets->dst_ipv4 || !packets->payload_len || !packets->send_time_ns || !status ||
         !deliver_time_ns || !event_id || !send || (!table->path_key && (!table->latency_ns || !table->packet_loss))))
      throw Error(SG_ERR_INVALID_ARG, "null packet or output array");
    deliver_source_padded(ctx, hosts, table, round, packets, status, deliver_time_ns, event_id, host_owner, n_ranks,
                          cap, send_padded, send, (unsigned long long*)xrow);
  });
}

int32_t sg_deliver_bucket_padded(sg_ctx* ctx, const sg_record* recv_padded, uint32_t n_ranks, uint32_t cap,
                                 const uint64_t* xall, uint32_t rank, const uint32_t* host_local, uint32_t n_hosts,
                                 uint32_t n_local_hosts, uint32_t* dst_order, uint32_t* dst_offsets,
                                 sg_round_stats* stats, uint32_t* recv_counts, uint32_t* pair_max) {
  return sg::guarded(ctx, [&] {
    using namespace sg;
    if (!recv_padded || !xall || !host_local || !dst_order || !dst_offsets)
      throw Error(SG_ERR_INVALID_ARG, "null argument");
    if (n_ranks == 0 || n_ranks > MAX_RANKS || rank >= n_ranks || cap == 0)
      throw Error(SG_ERR_INVALID_ARG, "bad n_ranks / rank / cap");
    deliver_bucket_padded(ctx, recv_padded, n_ranks, cap, (const unsigned long long*)xall, rank, host_local, n_hosts,
                          n_local_hosts, dst_order, dst_offsets, stats, recv_counts, pair_max);
  });
}

int32_t sg_deliver_pad_to_compact(sg_ctx* ctx, const sg_record* send_padded, uint32_t n_ranks, uint32_t cap,
                                  const uint64_t* xrow, sg_record* send) {
  return sg::guarded(ctx, [&] {
    using namespace sg;
    if (!send_padded || !xrow || !send || n_ranks == 0 || n_ranks > MAX_RANKS || cap == 0)
      throw Error(SG_ERR_INVALID_ARG, "bad argument");
    const size_t total = (size_t)n_ranks * cap;
    hipLaunchKernelGGL(k_pad_to_compact, dim3(grid_for(total, 256, 8192)), dim3(256), 0, ctx->stream, send_padded,
                       cap, (const unsigned long long*)xrow, n_ranks, send);
    SG_CHECK_LAUNCH();
  });
}

uint64_t* sg_hosts_event_ctr(sg_hosts* hosts) { return hosts ? hosts->ctr : nullptr; }

int32_t sg_table_pack(sg_ctx* ctx, const sg_table* table, uint64_t* out_key, uint32_t* out_packable) {
  return sg::guarded(ctx, [&] {
    using namespace sg;
    if (!table || !out_packable) throw Error(SG_ERR_INVALID_ARG, "null argument");
    const size_t cells = (size_t)table->n_rows * table->n_cols;
    if (cells && (!out_key || !table->latency_ns || !table->packet_loss))
      throw Error(SG_ERR_INVALID_ARG, "null table or output array");
    table_pack(ctx, table, cells, out_key, out_packable);
  });
}

int32_t sg_deliver_bucket(sg_ctx* ctx, const sg_record* recv, uint32_t n_records, const uint32_t* host_local,
                          uint32_t n_hosts, uint32_t n_local_hosts, uint32_t* dst_order, uint32_t* dst_offsets) {
  return sg::guarded(ctx, [&] {
    using namespace sg;
    if (!host_local || !dst_offsets || (n_records && (!recv || !dst_order)))
      throw Error(SG_ERR_INVALID_ARG, "null argument");
    deliver_bucket(ctx, recv, n_records, host_local, n_hosts, n_local_hosts, dst_order, dst_offsets);
  });
}

}  // extern "C"
