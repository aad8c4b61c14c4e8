// sg_sssp.hip -- per-source shortest paths with the distance row resident in LDS.
//
// Replaces, for graphs whose node count fits a CU's LDS (about 11k nodes), the
// per-source petgraph::algo::dijkstra of NetworkGraph::compute_shortest_paths
// (graph/mod.rs:190-208).  One workgroup owns one source row: its keys live in
// LDS for the whole search, the graph's out-arcs are read from L2 (one 12-B
// record per relaxation), and the finished row is written straight into the
// caller's row-major table.
//
// Why not the batched-source slab kernel (sg_routing.hip k_relax_w2) here: a
// 64-source batch gathers whole 512-B rows, and Bellman-Ford re-gathers a row
// whenever any of its 64 sources improved it -- about 10x the n_used * arcs
// relaxations of Dijkstra at C3.  A per-source search relaxes only what its own
// frontier improved: with delta-stepping buckets about 1.05-1.4x Dijkstra's
// relaxations (SG_SSSP_DIAG reports it).
//
// Exactness.  Edge latency >= 1 ns (graph/mod.rs:105-107) and the f32 loss fold
// is monotone, so petgraph's Dijkstra result is the unique fixed point of the
// source-rooted relaxation key[v] = min(key[v], key[u] (+) w(u, v)) with the
// edge applied on the right (sg_device.h fold_loss); any relaxation order
// reaches it.  Keys whose latency saturates at LAT32_SAT (>= 4.29 s, or
// unreachable) are never propagated and flag the row for the wide kernel
// (sg_routing.hip run_wide), as in the slab kernel.
//
// Flagged key.  key = (latency u32 << 32) | (bits(loss) << 1) | dirty.  Loss is
// in [0, 1], so bits(loss) < 2^31 and the 64-bit integer order of the key is the
// PathProperties order (latency, then loss), the flag ranking last.  A candidate
// carries dirty = 1, so one 64-bit LDS atomic min both relaxes and tests the
// flag: the node improved iff the returned key's (latency, loss) is larger, and
// it must be queued iff the returned key was clean.  An equal candidate never
// replaces a key (its flag is 1, the stored one 0 or 1), so "improved" means
// strictly better.  A pop clears the flag with one atomic AND whose return value
// is the key to relax with; an improvement that lands after it finds the flag
// clear and queues the node again.
//
// Work order: an asynchronous work queue per workgroup, with delta-stepping
// buckets (bucket width `delta`; one workgroup barrier per bucket, none per hop).
//   * A node is dirty from an improvement until it is popped; a node that
//     becomes dirty with latency below `split` is also appended to the queue,
//     so the queue never holds a node twice.
//   * The queue is an LDS ring of u16 node ids with head / tail counters.  A
//     wave claims up to 64 entries (CAS on head), relaxes their out-arcs and
//     appends what it improved (add on tail, then the slot writes; a claimed
//     slot not yet written reads as EMPTY and is waited for).  `busy` counts the
//     waves holding claimed entries; head and busy share one 64-bit LDS word,
//     so a claim is one CAS and a failed claim attempt changes nothing.
//   * Quiescence (busy == 0 and head == tail, read in that order) is stable: no
//     entry appears without a busy wave.  Every wave then meets at a barrier;
//     the dirty nodes left are those at or beyond `split`.  split = (smallest
//     dirty latency) + delta, the dirty nodes below it are queued, and the
//     waves go on.  No dirty node left: the search is done.
//   * Relaxing a popped node: when the largest out-degree among the wave's
//     entries is at most LANE_DEG_MAX, each lane walks its own node's arcs, eight
//     loads in flight (no cross-lane bookkeeping on the dependent chain);
//     otherwise the wave expands the entries' arcs into consecutive slots
//     (owner by scatter + max-scan) and relaxes SSSP_K chunks of 64 at once.
//
// Bounds (ub_row / ub_w).  For an arc s -> s' whose row D[s'] is already in the
// table, w(s, s') + D[s'][v] is the latency of a real path from s, so it bounds
// D[s][v] from above.  A bounded search starts key[v] at (that bound + 1, loss
// 1.0, clean) instead of infinity: still above the optimum, so the fixed point
// and the proof above are unchanged, but every candidate slower than the bound
// loses its first atomic min and is never queued.  sg_routing.hip sssp_plan
// orders the rows in phases, one launch each, so the bound rows of a phase are
// final (an earlier launch) before any search reads them.  A one-launch variant
// with per-row flags (searches reading rows other workgroups had just published)
// was tried: with an L2 write-back before each flag it matched bit for bit and
// saved 3 %, without it the table came out wrong, so it was dropped.
//
// Exact seeds.  When the arc s -> s' has zero loss (bits(1f32 - loss) == 1.0f),
// the left fold from s over s -> s' followed by any path P from s' gives exactly
// P's fold from s' (fold(0, 1.0) = 0, then the same sequence of f32 ops), so
// (w(s, s') + D[s'][v].lat, D[s'][v].loss) is the exact key of a real path.
// Such keys start CLEAN (never queued).  Still exact: every key is a real path's
// value (>= the optimum), and along an optimal path s = v0, .., vk every vi ends
// at its optimum by induction -- either v(i-1) was popped holding its optimum and
// relaxed vi, or v(i-1) held its optimum from the start, i.e. an exact seed via
// some s'; then vi's seed via the same s' is at most w + (D[s'][v(i-1)] (+)
// w(v(i-1), vi)) = opt(vi), so vi also starts at its optimum.  The induction needs
// a seed for every node, so the plan sets SSSP_UB_EXACT only when every node is a
// used node, and a bound row flagged for the wide kernel seeds bounds only.  A
// node reached optimally through an exactly seeded neighbour row is never
// popped: its subtree drops out of the search.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "sg_device.h"
#include "sg_internal.h"

namespace sg {

constexpr int SSSP_THREADS = 1024;  // the largest workgroup (SG_SSSP_THREADS selects 512 or 1024)
constexpr int SSSP_WAVES = SSSP_THREADS / 64;
constexpr int SSSP_K = 4;            // expansion path: chunks of 64 arc slots a wave handles at once
constexpr int SSSP_KB = SSSP_KB_MAX;  // bound rows per bounded search (sg_routing.hip sssp_plan)
// static LDS of k_sssp_lds: ctl[8] + red[SSSP_WAVES] (u32), hb (u64), own[SSSP_WAVES][64 * SSSP_K] (u8),
// sink[64] (u64), s_ub[SSSP_KB][3] + s_nub (u32)
constexpr size_t SSSP_STATIC_LDS = 4 * (8 + SSSP_WAVES) + 16 + SSSP_WAVES * 64 * SSSP_K + 512 + 4 * (3 * SSSP_KB + 1) + 16;
// lane path: arcs a lane has in flight (template LA: 8 or 16, SG_SSSP_LANE_ARCS);
// used up to out-degree lane_deg_max (SG_SSSP_LANE_DEG, default 64; the arcs past LA arc-parallel)

constexpr size_t LDS_PER_CU = 160 * 1024;

constexpr uint64_t FKEY_INF = ((uint64_t)LAT32_SAT << 32) | ((uint64_t)0x3F800000u << 1);  // (SAT, 1.0), clean
__device__ __forceinline__ uint32_t fkey_lat(uint64_t k) { return (uint32_t)(k >> 32); }
__device__ __forceinline__ uint32_t fkey_loss_bits(uint64_t k) { return ((uint32_t)k >> 1) & 0x7FFFFFFFu; }
// key(u) (+) edge (graph/mod.rs:322-331), flagged dirty
// (the loss is in [0, 1], never -0.0: its bits are below 2^31, so the low word is one 32-bit
// shift-or and the high word is the latency itself -- no 64-bit shift, no carry)
__device__ __forceinline__ uint64_t frelax(uint64_t ku, uint32_t edge_lat, float edge_om) {
  const uint32_t lat = __builtin_elementwise_add_sat(fkey_lat(ku), edge_lat);
  const float loss = fold_loss(__uint_as_float(fkey_loss_bits(ku)), edge_om);
  return ((uint64_t)lat << 32) | (uint32_t)((__float_as_uint(loss) << 1) | 1u);
}

// Queue capacity: n + 1024 rounded up to 64.  At most n nodes are queued (one
// entry per dirty node) and at most 16 waves x 64 claimed slots are still being
// read, so a slot is never reused while its last entry is unread.  Slot of a
// counter c: c mod cap by a multiply-high and one correction (cap < 2^17).
__host__ __device__ inline uint32_t sssp_ring_cap(uint32_t n) { return (n + 1024 + 63) / 64 * 64; }
struct RingMod {
  uint32_t cap, m;  // m = floor(2^32 / cap)
  __device__ __forceinline__ uint32_t operator()(uint32_t c) const {
    uint32_t r = c - __umulhi(c, m) * cap;  // in [0, 2 cap)
    return r >= cap ? r - cap : r;
  }
};
constexpr uint16_t RING_EMPTY = 0xFFFF;

// Queue the flagged lanes' nodes (NK candidates per lane): one tail add per call.
// mq[c]: the wave's ballot of candidate c (wave-uniform masks, no per-lane bool kept)
template <int NK>
__device__ __forceinline__ void append_q(const uint64_t* mq, const uint32_t* v, uint16_t* ring, uint32_t* tail,
                                         const RingMod& slot_of, int lane) {
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t tot = 0;
#pragma unroll
  for (int c = 0; c < NK; c++) tot += (uint32_t)__popcll(mq[c]);
  if (!tot) return;
  uint32_t b = 0;
  if (lane == 0) b = atomicAdd(tail, tot);
  b = __builtin_amdgcn_readfirstlane(b);
#pragma unroll
  for (int c = 0; c < NK; c++) {
    if ((mq[c] >> lane) & 1ull) ring[slot_of(b + (uint32_t)__popcll(mq[c] & lt))] = (uint16_t)v[c];
    b += (uint32_t)__popcll(mq[c]);
  }
}

// LDS bytes the kernel needs for n nodes (dynamic part): keys, staged out-arc
// offsets, the queue ring.
size_t sssp_lds_bytes(uint32_t n) {
  return (size_t)n * 8 + (((size_t)n + 1) * 4 + 7) / 8 * 8 + (size_t)sssp_ring_cap(n) * 2;
}

// One workgroup per source row i in [row_begin, row_end): source used[i].
// out_arc: 3 u32 per out-arc (destination, latency clamped to LAT32_SAT,
// bits(1f32 - loss)), grouped by tail node (out_off).
// PART: 0 for a routing build, 1 for sg_routing_info_fill's row blocks (the same
// code; a separate symbol so per-kernel profiles do not mix whole builds with blocks)
// FLAG: one launch for the whole plan (rows in phase order), bound rows taken
// only once published -- see "Flagged rows" below; `done` (per row, zeroed by the
// plan) is 1 for a final row, 2 for a final row with saturated keys (bounds only).
constexpr int SSSP_SC1 = 16;  // buffer cache-policy bits: sc1 (gfx950), MI355X_MICROARCH.md's hand-off
template <bool COUNT, int NT, int LA, int PART, bool FLAG = false>
__global__ void __launch_bounds__(NT)
    k_sssp_lds(const uint32_t* __restrict__ out_off, const uint32_t* __restrict__ out_arc, uint32_t n,
               uint32_t n_arcs, const uint32_t* __restrict__ used, uint32_t n_used, uint32_t row_begin,
               uint32_t out_row0, const uint32_t* __restrict__ self_edge, const uint64_t* __restrict__ e_lat,
               const float* __restrict__ e_loss, uint64_t* __restrict__ out_lat, float* __restrict__ out_loss,
               uint32_t* __restrict__ sat_row, uint32_t delta, int vec_out, unsigned long long* __restrict__ work,
               unsigned long long* __restrict__ diag, uint32_t claim, uint32_t idle_sleep,
               uint32_t lane_deg_max, const uint32_t* __restrict__ blk_rows,
               const uint32_t* __restrict__ ub_row, const uint32_t* __restrict__ ub_w,
               uint32_t* __restrict__ item_ctr, uint32_t n_items, uint32_t spin_max,
               const uint32_t* __restrict__ plan_ctl, int plan_ph, uint32_t* __restrict__ done) {
  constexpr int NW = NT / 64;
  constexpr int AUX = FLAG ? SSSP_SC1 : 0;  // bound rows and the output: sc1 in the flagged launch
  if (plan_ctl) {  // a device-built plan (sg_plan.hip): this phase's rows and bound rows, its row count
    const uint32_t base = plan_ctl[2 * plan_ph];
    n_items = plan_ctl[2 * plan_ph + 1];
    blk_rows += base;
    if (ub_row) {
      ub_row += (size_t)base * SSSP_KB;
      ub_w += (size_t)base * SSSP_KB;
    }
  }
  extern __shared__ __align__(16) unsigned char smem[];
  const uint32_t cap = sssp_ring_cap(n);
  const RingMod slot_of{cap, (uint32_t)(0x100000000ull / cap)};
  unsigned long long* key = (unsigned long long*)smem;
  uint32_t* off = (uint32_t*)(key + n);  // out_off staged in LDS (n + 1)
  uint16_t* ring = (uint16_t*)(smem + (size_t)n * 8 + (((size_t)n + 1) * 4 + 7) / 8 * 8);
  __shared__ uint32_t ctl[8];  // TAIL
  constexpr int TAIL = 1;
  // (head << 32) | busy in one word: a claim advances head and counts its wave
  // busy in one CAS, so a failed claim attempt never touches busy
  __shared__ unsigned long long hb;
  __shared__ uint8_t own[NW][64 * SSSP_K];
  __shared__ uint32_t red[NW];
  __shared__ unsigned long long sink[64];  // per-lane no-op target of offer_all
  __shared__ uint32_t s_ub[SSSP_KB][3];     // the row's usable bound rows: row, latency, exact
  __shared__ uint32_t s_nub;
  __shared__ uint32_t s_sat;  // FLAG: a wave saw a saturated key in the row's output
  if (FLAG && threadIdx.x == 0) s_sat = 0u;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // Every global read of the setup is a buffer load whose out-of-range lanes read
  // 0 without a branch, issued in groups so that a thread has a group's loads in
  // flight at once (one round trip per group, not per element).
  constexpr uint32_t OOB = 0x80000000u;
  {  // out_off staged in LDS, once per workgroup (a persistent one keeps it for all its rows)
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)out_off, 0, (int)((n + 1) * 4u),
                                                                        0x00020000);
    constexpr int GO = 12;  // entries per thread per group: one group up to 12,287 nodes
    for (uint32_t v0 = tid; v0 <= n; v0 += GO * NT) {
      uint32_t to[GO];
#pragma unroll
      for (int g = 0; g < GO; g++) {
        const uint32_t v = v0 + g * NT;
        to[g] = __builtin_amdgcn_raw_buffer_load_b32(ro, v <= n ? v * 4u : OOB, 0, 0);
      }
#pragma unroll
      for (int g = 0; g < GO; g++)
        if (v0 + g * NT <= n) off[v0 + g * NT] = to[g];
    }
  }
  // Rows: one per workgroup, or (item_ctr set: persistent workgroups, one per
  // CU) claimed one after another from a counter the host zeroed
  // The next row is claimed while this one's output is written (its returning
  // atomic then overlaps the stores instead of starting the next row's setup);
  // give-ups happen only during a search, never with a claim outstanding.
  __shared__ uint32_t s_item;
  if (item_ctr && tid == 0) s_item = atomicAdd(item_ctr, 1u);
  for (uint32_t it = 0;; it++) {
    uint32_t bi;
    if (item_ctr) {
      __syncthreads();  // s_item written (first row: above; later rows: in the previous row's output)
      bi = s_item;
      if (bi >= n_items) break;
    } else {
      if (it) break;
      bi = blockIdx.x;
      if (bi >= n_items) break;
    }
    // COUNT diagnostics of the first 4096 rows: cycle stamps, pops, bucket advances, relaxations
    const bool dg = COUNT && diag && bi < 4096 && tid == 0;
    const unsigned long long c_start = dg ? clock64() : 0;
    uint32_t n_adv = 0, n_pops = 0;
    unsigned long long cyc_claim = 0, cyc_pop = 0, cyc_steps = 0;  // per wave, COUNT diagnostics
    const uint32_t row = blk_rows ? blk_rows[bi] : row_begin + bi;
    const uint32_t src = used[row];
    // Setup: the LDS queue and keys (out_off is staged once, before the row loop)
    for (uint32_t v = tid; v < n; v += NT) key[v] = FKEY_INF;
    for (uint32_t i = tid; i < cap; i += NT) ring[i] = RING_EMPTY;
    for (int i = tid; i < NW * 64 * SSSP_K; i += NT) (&own[0][0])[i] = 0;
    if (tid < 8) ctl[tid] = 0;
    if (tid == 0) hb = 0;
    if (ub_row && tid < 64) {
      // wave 0 lists the row's usable bound rows in LDS while the others initialise: a
      // row whose search gave up (sat_row 2) was never written, so it gives no bounds; a
      // saturated one (1) holds real paths but not its optimum everywhere: bounds only
      const uint32_t e = tid < SSSP_KB ? ub_row[(size_t)bi * SSSP_KB + tid] : ~0u;
      const uint32_t w = tid < SSSP_KB ? ub_w[(size_t)bi * SSSP_KB + tid] : 0u;
      const uint32_t srow = e & ~SSSP_UB_EXACT;
      uint32_t sf;
      if constexpr (FLAG) {  // one sc1 poll per bound row, no wait: an unpublished row gives no bounds
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)done, 0, 0x7FFFFFFF, 0x00020000);
        const uint32_t dn = __builtin_amdgcn_raw_buffer_load_b32(rd, e != ~0u ? (srow - row_begin) * 4u : 0x80000000u,
                                                                 0, SSSP_SC1);
        sf = dn == 1u ? 0u : dn == 2u ? 1u : 2u;
      } else {
        sf = e != ~0u ? sat_row[srow - row_begin] : 2u;
      }
      const bool on = sf != 2u;
      const uint64_t mk = __ballot(on);
      if (on) {
        const int at = __popcll(mk & ((1ull << tid) - 1));
        s_ub[at][0] = srow;
        s_ub[at][1] = w;
        s_ub[at][2] = (e & SSSP_UB_EXACT) && sf == 0u;
      }
      if (tid == 0) s_nub = (uint32_t)__popcll(mk);
    }
    __syncthreads();
    if (ub_row) {  // Bounds: keys start just above the shortest of up to SSSP_KB known paths (clean)
      const int nb = (int)s_nub;
      if (nb) {
        const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc((void*)used, 0, (int)(n_used * 4u),
                                                                            0x00020000);
        constexpr int G = 6;  // columns per thread per group
        for (uint32_t j0 = tid; j0 < n_used; j0 += G * NT) {
          uint32_t vv[G];
          uint64_t m[G], ex[G];
#pragma unroll
          for (int g = 0; g < G; g++) {
            const uint32_t j = j0 + g * NT;
            vv[g] = __builtin_amdgcn_raw_buffer_load_b32(ru, j < n_used ? j * 4u : OOB, 0, 0);
            m[g] = ex[g] = ~0ull;
          }
#pragma unroll 1
          for (int k = 0; k < nb; k += 2) {  // two bound rows' loads in flight together
            bool on[2], exact[2];
            uint32_t sr[2], w[2];
            __amdgpu_buffer_rsrc_t rl[2], rf[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
              on[u] = k + u < nb;
              sr[u] = on[u] ? s_ub[k + u][0] : 0u;
              w[u] = on[u] ? s_ub[k + u][1] : 0u;
              exact[u] = on[u] && s_ub[k + u][2];
              const size_t rb = on[u] ? (size_t)(sr[u] - out_row0) * n_used : 0;
              rl[u] = __builtin_amdgcn_make_buffer_rsrc((void*)(out_lat + rb), 0, (int)(on[u] ? n_used * 8u : 0u),
                                                        0x00020000);
              rf[u] = __builtin_amdgcn_make_buffer_rsrc((void*)(out_loss + rb), 0, (int)(exact[u] ? n_used * 4u : 0u),
                                                        0x00020000);
            }
            uint64_t l[2][G];
            uint32_t f[2][G];
#pragma unroll
            for (int u = 0; u < 2; u++)
#pragma unroll
              for (int g = 0; g < G; g++) {
                const uint32_t j = j0 + g * NT;
                const auto x = __builtin_amdgcn_raw_buffer_load_b64(rl[u], j < n_used ? j * 8u : OOB, 0, AUX);
                l[u][g] = ((uint64_t)x[1] << 32) | x[0];
                f[u][g] = __builtin_amdgcn_raw_buffer_load_b32(rf[u], j < n_used ? j * 4u : OOB, 0, AUX);
              }
#pragma unroll
            for (int u = 0; u < 2; u++)
#pragma unroll
              for (int g = 0; g < G; g++) {
                const uint32_t j = j0 + g * NT;
                const uint64_t ub = l[u][g] + w[u];  // w < 2^32: a wrap means >= 2^64
                if (!on[u] || j >= n_used || ub < w[u]) continue;
                m[g] = min(m[g], ub);
                if (exact[u] && ub < LAT32_SAT && j != sr[u])  // exact: the path s -> s' then D[s'][v]
                  ex[g] = min(ex[g], (ub << 32) | ((uint64_t)f[u][g] << 1));
              }
          }
#pragma unroll
          for (int g = 0; g < G; g++) {
            uint64_t kv = m[g] < LAT32_SAT - 1 ? ((m[g] + 1) << 32) | ((uint64_t)0x3F800000u << 1) : FKEY_INF;
            kv = min(kv, ex[g]);
            if (j0 + g * NT < n_used && kv != FKEY_INF) key[vv[g]] = kv;
          }
        }
      }
      __syncthreads();
    }
    const unsigned long long c_setup = dg ? clock64() : 0;
    if (tid == 0) {
      key[src] = 1ull;  // PathProperties::default(), dirty and queued
      ring[0] = (uint16_t)src;
      ctl[TAIL] = 1;
    }
    uint32_t split = delta;  // delta >= 1
    const __amdgpu_buffer_rsrc_t arcs = __builtin_amdgcn_make_buffer_rsrc((void*)out_arc, 0, (int)(n_arcs * 12u),
                                                                          0x00020000);
    uint32_t n_rel = 0;
    // a bound no correct search reaches (a bucket advance queues at least one
    // node, and a node is queued at most once per improvement); past it the row
    // is handed to the wide kernel instead of spinning
    const uint32_t max_adv = 4u * n + 64u;
    uint8_t* ow = own[wv];
    // spin budget per wave (sleeps of ~128 cycles): a safety valve against a
    // queue bug, never reached by a correct search; past it the wave leaves and
    // the row goes to the wide kernel
    uint32_t spins = 0;
    // Giving up (the safety valves below, never reached by a correct search):
    // the wave flags the row for the wide kernel, sets ctl[ABORT] and leaves the
    // kernel; every other wave of the workgroup leaves too, at its next claim or
    // after the quiescence barrier, so no wave waits at a barrier the others
    // will not reach, and a persistent workgroup takes no further rows (the
    // other workgroups claim them).
    constexpr int ABORT = 2;
    auto give_up = [&]() {
      if (lane == 0) {
        sat_row[row - row_begin] = 2u;  // never written: the wide kernel redoes it, and no search bounds by it
        // the workgroup's first wave to give up counts it out; when every persistent
        // workgroup has given up (none left to claim the rest), the last one flags the
        // rows none claimed.  (A workgroup that ends normally has seen every row claimed.)
        if (atomicExch(&ctl[ABORT], 1u) == 0u && item_ctr) {
          __threadfence();
          if (atomicAdd(&item_ctr[1], 1u) == gridDim.x - 1) {
            const uint32_t c = __hip_atomic_load(&item_ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (uint32_t i = min(c, n_items); i < n_items; i++)
              sat_row[(blk_rows ? blk_rows[i] : row_begin + i) - row_begin] = 2u;
          }
        }
      }
    };
    auto ld = [](uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    // relax NK candidates into key[v[c]]; app[c]: the ballot of the lanes whose v[c] became dirty below split (to
    // be queued).  Branch-free, so the NK LDS atomics issue back to back and share
    // one wait: a lane with no candidate (or a saturated one, never propagated)
    // offers ~0 to its own sink word, a no-op.  (With one branch per candidate the
    // compiler waited for each atomic's return before issuing the next.)
    auto offer_all = [&](auto nk, const bool* valid, const uint32_t* v, const uint64_t* cand, uint64_t* app) {
      constexpr int NK = decltype(nk)::value;
      uint64_t cd[NK], old[NK];
      bool okk[NK];
#pragma unroll
      for (int c = 0; c < NK; c++) {
        const bool ok = valid[c] && fkey_lat(cand[c]) != LAT32_SAT;
        okk[c] = ok;
        // (no select of the offered value: a lane without a candidate offers whatever it holds
        // to its own sink word, whose value nothing reads)
        cd[c] = cand[c];
        old[c] = __hip_atomic_fetch_min(ok ? &key[v[c]] : &sink[lane], (unsigned long long)cd[c], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      // keep the scheduler from pulling a use of old[] between the atomics
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < NK; c++)
        // improved and was clean: a clean old key (flag 0) is above the candidate (flag 1) iff its
        // (latency, loss) is larger -- one 64-bit compare, no shifts
        // (the i1 ballot: the condition's lane mask as is, not a 0/1 VGPR compared back to a mask)
        app[c] = __builtin_amdgcn_ballot_w64(okk[c] && !((uint32_t)old[c] & 1u) && old[c] > cd[c] &&
                                             fkey_lat(cd[c]) < split);
    };
    __syncthreads();

    for (;;) {
      // ---- claim up to `claim` queued entries
      const unsigned long long tc0 = (COUNT && diag) ? clock64() : 0;
      uint32_t h = 0, k = 0;
      if (lane == 0) {
        for (;;) {
          const unsigned long long w = __hip_atomic_load(&hb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const uint32_t hh = (uint32_t)(w >> 32), t = ld(&ctl[TAIL]);
          if (t == hh) break;
          const uint32_t kk = min(claim, t - hh);
          const unsigned long long nw = ((unsigned long long)(hh + kk) << 32) | ((w & 0xFFFFFFFFull) + 1);
          if (atomicCAS(&hb, w, nw) == w) {
            h = hh;
            k = kk;
            break;
          }
        }
      }
      h = __builtin_amdgcn_readfirstlane(h);
      k = __builtin_amdgcn_readfirstlane(k);
      if (__builtin_amdgcn_readfirstlane(ld(&ctl[ABORT]))) goto wave_exit;  // another wave gave up
      if (!k) {
        uint32_t q = 0;
        if (lane == 0) {
          const unsigned long long w = __hip_atomic_load(&hb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __atomic_signal_fence(__ATOMIC_SEQ_CST);  // (head, busy) before tail (see header)
          q = (w & 0xFFFFFFFFull) == 0 && (uint32_t)(w >> 32) == ld(&ctl[TAIL]);
        }
        if (!__builtin_amdgcn_readfirstlane(q)) {
          if (++spins > spin_max) {
            give_up();
            goto wave_exit;
          }
          for (uint32_t z = 0; z < idle_sleep; z++) __builtin_amdgcn_s_sleep(8);  // ~512 cycles each
          __builtin_amdgcn_s_sleep(2);
          continue;
        }
        // ---- quiescent: every wave is here.  Next bucket, or done.
        __syncthreads();
        if (ld(&ctl[ABORT])) goto wave_exit;  // a wave gave up before this barrier (uniform: no wave is spinning now)
        // one bucket (split = LAT32_SAT, the default): every node that became dirty was
        // queued, so a quiescent queue means nothing is dirty -- no key scan needed
        if (split >= LAT32_SAT) break;
        uint32_t m = LAT32_SAT;
        for (uint32_t v = tid; v < n; v += NT) {
          const uint64_t kv = key[v];
          if (kv & 1ull) m = min(m, fkey_lat(kv));
        }
        for (int d = 32; d > 0; d >>= 1) m = min(m, (uint32_t)__shfl_xor(m, d));
        if (lane == 0) red[wv] = m;
        __syncthreads();
        m = red[0];
        for (int w = 1; w < NW; w++) m = min(m, red[w]);
        if (m == LAT32_SAT) break;  // nothing dirty (saturated keys are never marked dirty)
        if (++n_adv > max_adv) {  // every wave is here together
          give_up();
          goto wave_exit;
        }
        split = m + delta >= m ? min(m + delta, LAT32_SAT) : LAT32_SAT;
        for (uint32_t v0 = wv * 64; v0 < n; v0 += NT) {  // queue the dirty nodes below split
          const uint32_t v = v0 + lane;
          uint64_t kv = v < n ? key[v] : 0ull;
          const bool q2 = (kv & 1ull) && fkey_lat(kv) < split;
          const uint64_t m2 = __ballot(q2);
          append_q<1>(&m2, &v, ring, &ctl[TAIL], slot_of, lane);
        }
        __syncthreads();
        continue;
      }
      if (COUNT) n_pops++;
      const unsigned long long tc1 = (COUNT && diag) ? clock64() : 0;
      // ---- pop the claimed entries (a slot claimed before its writer stored it reads EMPTY)
      const bool on = lane < (int)k;
      uint32_t u = 0, a0 = 0, a1 = 0;
      uint64_t ku = 0;
      bool stuck = false;
      if (on) {
        volatile uint16_t* slot = &ring[slot_of(h + lane)];
        uint16_t x;
        uint32_t sp = 0;
        while ((x = *slot) == RING_EMPTY && ++sp < spin_max) __builtin_amdgcn_s_sleep(0);
        stuck = x == RING_EMPTY;
        *slot = RING_EMPTY;
        u = stuck ? src : x;
        a0 = off[u];
        a1 = off[u + 1];
        // clear the dirty flag; the returned key is the one to relax with (see header)
        ku = __hip_atomic_fetch_and(&key[u], ~1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & ~1ull;
      }
      if (__any(stuck)) {
        give_up();
        goto wave_exit;
      }
      const uint32_t deg = a1 - a0;
      const uint32_t dmax = __builtin_amdgcn_readlane(wave_incl_max(deg), 63);
      const unsigned long long tc2 = (COUNT && diag) ? clock64() : 0;
      // arcs [ea0, ea0 + edeg) of each lane's node, arc-parallel: the wave's arcs in consecutive
      // slots, KX chunks of 64 at once (owner lane by scatter + max-scan)
      auto expand = [&](auto kx, uint32_t ea0, uint32_t edeg) {
        constexpr int KX = decltype(kx)::value;
        const uint32_t incl = wave_incl_sum(edeg);
        const uint32_t base = incl - edeg;
        const uint32_t T = __builtin_amdgcn_readlane(incl, 63);
        if (COUNT) n_rel += T;
        uint32_t carry = 0;  // 1 + the owner lane of the previous slot
        for (uint32_t t0 = 0; t0 < T; t0 += 64 * KX) {
          // owner lane of each slot: heads scatter 1 + their lane at their first slot, a max-scan fills the rest
          if (edeg && base >= t0 && base - t0 < 64u * KX) ow[base - t0] = (uint8_t)(lane + 1);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          uint32_t v[KX], lat[KX], om[KX], o[KX];
          bool valid[KX];
          uint64_t app[KX];
#pragma unroll
          for (int c = 0; c < KX; c++) {
            const uint32_t hd = ow[c * 64 + lane];
            ow[c * 64 + lane] = 0;
            const uint32_t mx = max(wave_incl_max(hd), carry);
            carry = __builtin_amdgcn_readlane(mx, 63);
            o[c] = mx - 1;
          }
#pragma unroll
          for (int c = 0; c < KX; c++) {
            const uint32_t sl = t0 + c * 64 + lane;
            valid[c] = sl < T;
            const uint32_t a = __shfl(ea0, (int)o[c]) + sl - __shfl(base, (int)o[c]);
            const auto r = __builtin_amdgcn_raw_buffer_load_b96(arcs, valid[c] ? a * 12u : 0x80000000u, 0, 0);
            v[c] = r[0];
            lat[c] = r[1];
            om[c] = r[2];
          }
          uint64_t cand[KX];
#pragma unroll
          for (int c = 0; c < KX; c++) {
            const uint32_t klo = __shfl((uint32_t)ku, (int)o[c]), khi = __shfl((uint32_t)(ku >> 32), (int)o[c]);
            cand[c] = frelax(((uint64_t)khi << 32) | klo, lat[c], __uint_as_float(om[c]));
          }
          offer_all(std::integral_constant<int, KX>(), valid, v, cand, app);
          append_q<KX>(app, v, ring, &ctl[TAIL], slot_of, lane);
        }
      };
      if (dmax <= lane_deg_max) {
        // ---- lane path: each lane walks its node's first LA arcs (LA loads in flight); the arcs
        // past them (nodes of degree > LA only) go arc-parallel like the expansion path.  At C3
        // (mean degree 8, a wave's largest ~14) a second round of LA slots per lane was mostly
        // idle lanes: 3.10 -> 2.83 ms (profiles/r05/ab_sssp_hybrid_r6x.txt)
        if (COUNT) n_rel += __builtin_amdgcn_readlane(wave_incl_sum(min(deg, (uint32_t)LA)), 63);
        {
          constexpr uint32_t j0 = 0;
          uint32_t v[LA], lat[LA], om[LA];
          bool valid[LA];
          uint64_t app[LA];
#pragma unroll
          for (int c = 0; c < LA; c++) {
            valid[c] = j0 + c < deg;
            const auto r = __builtin_amdgcn_raw_buffer_load_b96(arcs, valid[c] ? (a0 + j0 + c) * 12u : 0x80000000u,
                                                                0, 0);
            v[c] = r[0];
            lat[c] = r[1];
            om[c] = r[2];
          }
          uint64_t cand[LA];
#pragma unroll
          for (int c = 0; c < LA; c++) cand[c] = frelax(ku, lat[c], __uint_as_float(om[c]));
          offer_all(std::integral_constant<int, LA>(), valid, v, cand, app);
          append_q<LA>(app, v, ring, &ctl[TAIL], slot_of, lane);
        }
        if (dmax > (uint32_t)LA)  // the arcs past each node's first LA, arc-parallel
          expand(std::integral_constant<int, 1>(), a0 + LA, deg > (uint32_t)LA ? deg - LA : 0u);
      } else {
        // ---- expansion path (high out-degree): arcs of the 64 entries in consecutive slots
        expand(std::integral_constant<int, SSSP_K>(), a0, deg);
      }
      // release the claim after this wave's appends (LDS keeps a wave's operations in order)
      if (lane == 0) atomicSub(&hb, 1ull);
      if (COUNT && diag) {
        const unsigned long long tc3 = clock64();
        cyc_claim += tc1 - tc0;
        cyc_pop += tc2 - tc1;
        cyc_steps += tc3 - tc2;
      }
    }
    if (COUNT && lane == 0 && n_rel) atomicAdd(&work[bi & 63], (unsigned long long)n_rel);
    if (COUNT && diag && bi < 4096 && lane == 0) {
      if (n_rel) atomicAdd(&diag[bi * 8 + 4], (unsigned long long)n_rel);
      if (n_pops) atomicAdd(&diag[bi * 8 + 2], (unsigned long long)n_pops);
      atomicAdd(&diag[bi * 8 + 5], cyc_claim);
      atomicAdd(&diag[bi * 8 + 6], cyc_pop);
      atomicAdd(&diag[bi * 8 + 7], cyc_steps);
    }
    const unsigned long long c_search = dg ? clock64() : 0;

    // ---- write the row: columns in used order, diagonal = the raw self-loop (graph/mod.rs:210-217)
    __syncthreads();  // every thread has read s_item (at the row's start) before it is written again
    if (item_ctr && tid == 0) s_item = atomicAdd(item_ctr, 1u);  // the next row (see the row loop)
    const size_t orow = (size_t)(row - out_row0) * n_used;
    bool sat = false;
    // the row's output: nontemporal 16-B stores; in the flagged launch sc1 (write-through) stores,
    // which the later rows' sc1 loads read across XCDs (MI355X_MICROARCH.md hand-off protocol)
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t wl = __builtin_amdgcn_make_buffer_rsrc((void*)(out_lat + orow), 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t wf = __builtin_amdgcn_make_buffer_rsrc((void*)(out_loss + orow), 0, 0x7FFFFFFF, 0x00020000);
    auto st_lat2 = [&](uint32_t j, uint64_t a, uint64_t b) {
      if constexpr (FLAG) {
        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128((v4){(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)},
                                               wl, j * 8u, 0, SSSP_SC1);
      } else {
        __builtin_nontemporal_store((u64x2){a, b}, (u64x2*)&out_lat[orow + j]);
      }
    };
    auto st_loss4 = [&](uint32_t j, float a, float b, float c, float d) {
      if constexpr (FLAG) {
        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128((v4){__float_as_uint(a), __float_as_uint(b), __float_as_uint(c),
                                                    __float_as_uint(d)}, wf, j * 4u, 0, SSSP_SC1);
      } else {
        __builtin_nontemporal_store((f32x4){a, b, c, d}, (f32x4*)&out_loss[orow + j]);
      }
    };
    auto entry = [&](uint32_t j, uint64_t& l, float& f) {
      if (j == row) {
        const uint32_t e = self_edge[used[j]];
        l = e_lat[e];
        f = e_loss[e];
      } else {
        const uint64_t kk = key[used[j]];
        sat |= fkey_lat(kk) == LAT32_SAT;
        l = fkey_lat(kk);
        f = __uint_as_float(fkey_loss_bits(kk));
      }
    };
    if (vec_out) {  // n_used % 4 == 0, 16-B aligned rows: 16-B stores
      // Every global read of the output comes before its first store: the columns'
      // node ids (16-B loads, OU per thread) and the diagonal's raw self-loop.  (Read
      // inside the loop, each one waited behind the thread's earlier stores, since the
      // vector-memory counter covers both.)
      constexpr int OU = 4;
      const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc((void*)used, 0, (int)(n_used * 4u),
                                                                          0x00020000);
      // the column indices are computed here, per row, from an opaque copy of tid: hoisted
      // out of the row loop, the compiler kept (and spilled) them across the whole search
      uint32_t tt = (uint32_t)tid;
      asm volatile("" : "+v"(tt));
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      u32x4 uv[OU];
#pragma unroll
      for (int k = 0; k < OU; k++) {
        const uint32_t j = (tt + (uint32_t)k * NT) * 4;
        uv[k] = __builtin_amdgcn_raw_buffer_load_b128(ru, j < n_used ? j * 4u : OOB, 0, 0);
      }
      const uint32_t de = self_edge[src];
      const uint64_t d_lat = e_lat[de];
      const float d_loss = e_loss[de];
      auto cell = [&](uint32_t j, uint32_t vj, uint64_t& l, float& f) {
        const uint64_t kk = key[vj];
        const bool diag = j == row;
        sat |= !diag && fkey_lat(kk) == LAT32_SAT;
        l = diag ? d_lat : (uint64_t)fkey_lat(kk);
        f = diag ? d_loss : __uint_as_float(fkey_loss_bits(kk));
      };
#pragma unroll
      for (int k = 0; k < OU; k++) {
        const uint32_t j = (tt + (uint32_t)k * NT) * 4;
        if (j < n_used) {
          uint64_t l0, l1, l2, l3;
          float f0, f1, f2, f3;
          cell(j, uv[k][0], l0, f0);
          cell(j + 1, uv[k][1], l1, f1);
          cell(j + 2, uv[k][2], l2, f2);
          cell(j + 3, uv[k][3], l3, f3);
          st_lat2(j, l0, l1);
          st_lat2(j + 2, l2, l3);
          st_loss4(j, f0, f1, f2, f3);
        }
      }
      for (uint32_t j = (tt + OU * NT) * 4; j < n_used; j += NT * 4) {  // past OU x NT x 4 columns
        uint64_t l0, l1, l2, l3;
        float f0, f1, f2, f3;
        entry(j, l0, f0);
        entry(j + 1, l1, f1);
        entry(j + 2, l2, f2);
        entry(j + 3, l3, f3);
        st_lat2(j, l0, l1);
        st_lat2(j + 2, l2, l3);
        st_loss4(j, f0, f1, f2, f3);
      }
    } else {
      for (uint32_t j = tid; j < n_used; j += NT) {
        uint64_t l;
        float f;
        entry(j, l, f);
        if constexpr (FLAG) {
          __builtin_amdgcn_raw_buffer_store_b64((uint32_t __attribute__((ext_vector_type(2)))){(uint32_t)l,
                                                                                              (uint32_t)(l >> 32)},
                                                wl, j * 8u, 0, SSSP_SC1);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(f), wf, j * 4u, 0, SSSP_SC1);
        } else {
          out_lat[orow + j] = l;
          out_loss[orow + j] = f;
        }
      }
    }
    if (__any(sat) && lane == 0) {
      sat_row[row - row_begin] = 1u;
      if (FLAG) s_sat = 1u;
    }
    if (dg) {
      diag[bi * 8 + 0] = c_search - c_start;
      diag[bi * 8 + 1] = clock64() - c_search;
      diag[bi * 8 + 3] = n_adv | ((c_setup - c_start) << 24);  // bucket advances | setup cycles
    }
    if constexpr (FLAG) {
      // Flagged rows: every wave waits for its sc1 stores, then one lane publishes the row
      // (sc1 flag store behind the barrier: MI355X_MICROARCH.md hand-off table, first row)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)done, 0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(s_sat ? 2u : 1u, rd, (row - row_begin) * 4u, 0, SSSP_SC1);
        s_sat = 0u;
      }
    }
    __syncthreads();  // the next row reuses the LDS
  }
wave_exit:;
  // (An earlier version counted every wave out with one device atomic at exit: 4,096
  // atomics on one word at the end of each launch cost ~0.1 ms.)
}

bool sssp_lds_fits(uint32_t n) {
  if (n == 0 || n >= RING_EMPTY) return false;  // u16 queue entries
  return sssp_lds_bytes(n) + SSSP_STATIC_LDS <= LDS_PER_CU;
}

// Rows [row_begin, row_end) of the table (out_* device, row-major from out_row0).
// sat_row (device, row_end - row_begin u32) receives 1 for rows needing the wide kernel.
void launch_sssp_lds(sg_ctx* ctx, const uint32_t* out_off, const uint32_t* out_arc, uint32_t n, uint32_t n_arcs,
                     const uint32_t* d_used, uint32_t n_used, uint32_t row_begin, uint32_t row_end,
                     const uint32_t* self_edge, const uint64_t* e_lat, const float* e_loss, uint64_t* out_lat,
                     float* out_loss, uint32_t* sat_row, uint32_t delta, unsigned long long* work,
                     unsigned long long* diag, const uint32_t* blk_rows, uint32_t n_blk, const uint32_t* ub_row,
                     const uint32_t* ub_w, const uint32_t* plan_ctl, int plan_ph, uint32_t* plan_ctr,
                     uint32_t* done) {
  const size_t lds = sssp_lds_bytes(n);
  if (!sssp_lds_fits(n)) throw Error(SG_ERR_INVALID_ARG, "graph too large for the LDS-resident search");
  if ((uint64_t)n_arcs * 12 >= (1ull << 31)) throw Error(SG_ERR_INVALID_ARG, "too many arcs for 32-bit offsets");
  // entries a wave claims at once (SG_SSSP_CLAIM, 1..64)
  const char* cs = getenv("SG_SSSP_CLAIM");
  const uint32_t claim = (uint32_t)std::min(64, std::max(1, cs && *cs ? atoi(cs) : 64));
  const int vec = n_used % 4 == 0 && ((uintptr_t)out_lat & 15) == 0 && ((uintptr_t)out_loss & 15) == 0;
  // with a device plan (plan_ctl), n_blk bounds the phase's row count, which only the device knows
  const uint32_t rows = blk_rows ? n_blk : row_end - row_begin;
  if (!rows) return;
  const char* ts = getenv("SG_SSSP_THREADS");
  const int nt = ts && atoi(ts) == 512 ? 512 : 1024;
  const char* ss = getenv("SG_SSSP_SLEEP");  // idle back-off, units of ~512 cycles
  const uint32_t idle_sleep = ss && *ss ? (uint32_t)std::max(0, atoi(ss)) : 0u;
  const char* ls = getenv("SG_SSSP_LANE_DEG");
  // (with the remainder arc-parallel, every wave takes the lane path unless SG_SSSP_LANE_DEG
  // lowers it: C3 2.83 ms at 16, 2.79 at 24 and 64)
  const uint32_t lane_deg = ls && *ls ? (uint32_t)std::max(0, atoi(ls)) : 64u;
  const char* la = getenv("SG_SSSP_LANE_ARCS");
  const int la16 = la && atoi(la) == 16, la4 = la && atoi(la) == 4;
  // One persistent workgroup per CU claims rows from a counter: out_off is
  // staged once per CU instead of once per row, and no workgroup is launched and
  // torn down per row.  C3: 3.92 -> 3.54 ms (same box).  SG_SSSP_PERSIST=0: a
  // workgroup per row.
  const char* ps = getenv("SG_SSSP_PERSIST");
  const bool persist = done || (!(ps && ps[0] == '0') && (rows > (uint32_t)ctx->n_cu || plan_ctl));
  // spin budget per wave (sleeps of ~128 cycles): a safety valve against a queue
  // bug, never reached by a correct search; SG_SSSP_SPIN_MAX (tests) lowers it so
  // that searches give up and their rows take the wide kernel
  const char* sm = getenv("SG_SSSP_SPIN_MAX");
  const uint32_t spin_max = sm && *sm ? (uint32_t)std::max(1, atoi(sm)) : (1u << 22);
  // [claims, waves done] (sg_sssp.hip wave_exit); a device plan's counters are zeroed by the plan kernel
  uint32_t* item_ctr = nullptr;
  if (persist && plan_ctr) {
    item_ctr = plan_ctr;
  } else if (persist) {
    item_ctr = ctx->r_items.get<uint32_t>(2);
    SG_HIP(hipMemsetAsync(item_ctr, 0, 8, ctx->stream));
  }
  const uint32_t grid = persist ? (uint32_t)ctx->n_cu : rows;
  auto go = [&](auto kern) {
    SG_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(LDS_PER_CU - SSSP_STATIC_LDS)));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(nt), lds, ctx->stream, out_off, out_arc, n, n_arcs, d_used, n_used,
                       row_begin, row_begin, self_edge, e_lat, e_loss, out_lat, out_loss, sat_row, delta, vec, work,
                       diag, claim, idle_sleep, lane_deg, blk_rows, ub_row, ub_w, item_ctr, rows, spin_max, plan_ctl,
                       plan_ph, done);
  };
  if (done) {  // the flagged one-launch plan (the default kernel shape only)
    if (work) go(k_sssp_lds<true, 1024, 8, 0, true>);
    else if (ctx->in_fill) go(k_sssp_lds<false, 1024, 8, 1, true>);
    else go(k_sssp_lds<false, 1024, 8, 0, true>);
  } else if (work) {
    if (nt == 512) go(k_sssp_lds<true, 512, 8, 0>);
    else if (la16) go(k_sssp_lds<true, 1024, 16, 0>);
    else go(k_sssp_lds<true, 1024, 8, 0>);
  } else if (ctx->in_fill) {
    go(k_sssp_lds<false, 1024, 8, 1>);
  } else {
    if (nt == 512) go(k_sssp_lds<false, 512, 8, 0>);
    else if (la16) go(k_sssp_lds<false, 1024, 16, 0>);
    else if (la4) go(k_sssp_lds<false, 1024, 4, 0>);
    else go(k_sssp_lds<false, 1024, 8, 0>);
  }
  SG_CHECK_LAUNCH();
}

}  // namespace sg
