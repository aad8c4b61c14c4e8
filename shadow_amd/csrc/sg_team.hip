// sg_team.hip -- per-source shortest paths for graphs too large for one CU's LDS:
// a team of K workgroups (one per CU) holds one source row, each member the keys
// of 1/K of the nodes in its LDS.
//
// The reference runs petgraph's Dijkstra per used source (graph/mod.rs:190-200),
// work-efficient at any size.  sg_sssp.hip's search keeps a whole row of keys in
// one CU's LDS, which ends at about 11k nodes; past it the batched-source slab
// kernel (k_relax_w2) re-relaxes a 64-source batch's rows whenever any of its
// sources improved them -- about 10x Dijkstra's relaxations at C5's 50k nodes.
// Here the row is split instead: member m of a team owns nodes [m P, (m + 1) P)
// (P = ceil(n / K)) and their keys (the flagged keys of sg_sssp.hip: latency <<
// 32 | bits(loss) << 1 | dirty).  The search runs in supersteps:
//   1. local phase: the LDS work-queue search of sg_sssp.hip over the member's
//      own nodes and the arcs between them, to quiescence.  A popped node with
//      arcs to other members is marked in an LDS bitmap;
//   2. remote pass: every marked node, with its key as the local phase left it,
//      relaxes its arcs to other members once; each candidate is a 16-byte
//      message (target's local index, candidate key) appended to the block of
//      its target member in the team's outbox (HBM, written sc1: write-through);
//   3. exchange: the member publishes its per-target counts and arrives at the
//      team's barrier (one agent-scope counter); after it, every member reads
//      every count, and a superstep in which nobody sent anything ends the row
//      (all members read the same counts, so they agree);
//   4. apply: the member offers every message addressed to it to its keys (the
//      same 64-bit LDS atomic min as a local relaxation) and queues what
//      improved; then the next superstep.
// A node relaxes its remote arcs at most once per superstep, so a block never
// holds more messages than arcs between its two members (its capacity).
// Hand-offs follow MI355X_MICROARCH.md's measured sc1 protocol: every message
// and count is stored sc1 and loaded sc1, every storing wave waits for its
// stores (vmcnt(0)) before the workgroup barrier behind which one lane adds to
// the team's counter, and readers poll that counter with sc1 loads.  Any
// placement works (members on different XCDs included).
//
// Exactness is sg_sssp.hip's argument unchanged: every key is a real path's,
// the relaxation applies the edge on the right (fold_loss), and any order of
// relaxations reaches petgraph's fixed point.  Team membership is taken in
// order of arrival (a counter), so only workgroups that are running form teams;
// every wait has a budget, past which the team aborts, its rows are flagged (2)
// and the caller redoes them with the wide kernel.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "sg_device.h"
#include "sg_internal.h"

namespace sg {

namespace {

constexpr int TM_THREADS = 1024;
constexpr int TM_WAVES = TM_THREADS / 64;
constexpr int TM_LA = 8;            // arcs a lane has in flight
constexpr int TM_KMAX = 8;          // members per team
constexpr uint32_t TM_CTL_WORDS = 256;  // per team: row, arrive, abort, pad, counts[2][K][K]
constexpr uint16_t TM_EMPTY = 0xFFFF;
constexpr uint64_t TM_INF = ((uint64_t)LAT32_SAT << 32) | ((uint64_t)0x3F800000u << 1);  // (SAT, 1.0), clean
constexpr uint32_t TM_ROW_END = 0xFFFFFFFFu;
constexpr int TM_SC1 = 16;  // buffer cache-policy bits: sc1 (gfx950), the write-through / L2-served hand-off
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr size_t TM_LDS = 160 * 1024;
constexpr size_t TM_STATIC_LDS = 4 * (8 + TM_WAVES) + 8 + 512 + 4 * (2 * TM_KMAX * TM_KMAX + TM_KMAX + 4) + 64;

__device__ __forceinline__ uint32_t tk_lat(uint64_t k) { return (uint32_t)(k >> 32); }
__device__ __forceinline__ uint32_t tk_loss_bits(uint64_t k) { return ((uint32_t)k >> 1) & 0x7FFFFFFFu; }
__device__ __forceinline__ uint64_t tk_relax(uint64_t ku, uint32_t edge_lat, float edge_om) {
  const uint32_t lat = __builtin_elementwise_add_sat(tk_lat(ku), edge_lat);
  const float loss = fold_loss(__uint_as_float(tk_loss_bits(ku)), edge_om);
  return ((uint64_t)lat << 32) | ((uint64_t)__float_as_uint(loss) << 1) | 1ull;
}

__host__ __device__ inline uint32_t tm_ring_cap(uint32_t p) { return (p + 1024 + 63) / 64 * 64; }
struct TmRing {
  uint32_t cap, m;
  __device__ __forceinline__ uint32_t operator()(uint32_t c) const {
    uint32_t r = c - __umulhi(c, m) * cap;
    return r >= cap ? r - cap : r;
  }
};

size_t tm_lds_bytes(uint32_t p) { return (size_t)p * 8 + (size_t)tm_ring_cap(p) * 2 + ((size_t)p + 31) / 32 * 4; }

// Per node: its out-arcs to its own member first, then the rest (team_mid = the
// local count); the (member, member) arc counts size the outbox blocks.
__global__ void k_team_arcs(const uint32_t* __restrict__ out_off, const uint32_t* __restrict__ out_arc, uint32_t n,
                            uint32_t P, uint32_t K, uint32_t* __restrict__ team_arc, uint32_t* __restrict__ team_mid,
                            uint32_t* __restrict__ pair_cnt) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n) return;
  const uint32_t m = u / P, a0 = out_off[u], a1 = out_off[u + 1];
  uint32_t lo = a0, hi = a1;
  for (uint32_t a = a0; a < a1; a++) {
    const uint32_t v = out_arc[3 * (size_t)a], l = out_arc[3 * (size_t)a + 1], om = out_arc[3 * (size_t)a + 2];
    const uint32_t d = v / P;
    const uint32_t at = d == m ? lo++ : --hi;
    team_arc[3 * (size_t)at] = v;
    team_arc[3 * (size_t)at + 1] = l;
    team_arc[3 * (size_t)at + 2] = om;
    if (d != m) atomicAdd(&pair_cnt[m * K + d], 1u);
  }
  team_mid[u] = lo - a0;
}

struct TeamArgs {
  const uint32_t* out_off;   // n + 1
  const uint32_t* team_arc;  // 3 u32 per arc, own-member arcs first
  const uint32_t* team_mid;  // own-member arc count per node
  uint32_t n, n_arcs, P, K;
  const uint32_t* used;
  uint32_t n_used, row_begin;
  const uint32_t* mem_used;  // per member: the used indices j whose node it owns, ascending (stride n_used)
  const uint32_t* mem_n;     // their counts
  const uint32_t* self_edge;
  const uint64_t* e_lat;
  const float* e_loss;
  uint64_t* out_lat;
  float* out_loss;
  uint32_t* sat_row;
  uint32_t* rows_ctr;   // [0] next row index, [1] join counter
  uint32_t n_items;     // rows of this launch: row_begin + i
  uint32_t n_teams;
  uint32_t* team_ctl;   // n_teams x TM_CTL_WORDS
  uint4* outbox;        // n_teams x 2 x K x K x cap
  uint32_t cap;         // messages per (source, target) block
  uint32_t spin_max;
  unsigned long long* work;  // optional: relaxations (local and remote) and messages
  // a phase of the device plan (sg_plan.hip), or all null: rows row_begin + i
  const uint32_t* blk_rows;  // the plan's row list
  const uint32_t* ub_row;    // SSSP_KB_MAX bound rows per list position (SSSP_UB_EXACT: exact seeds)
  const uint32_t* ub_w;
  const uint32_t* plan_ctl;  // [2 ph] first list position, [2 ph + 1] rows of the phase
  int plan_ph;
};

__global__ void __launch_bounds__(TM_THREADS) k_sssp_team(TeamArgs a) {
  constexpr int NT = TM_THREADS;
  extern __shared__ __align__(16) unsigned char smem[];
  const uint32_t P = a.P, K = a.K;
  const uint32_t rcap = tm_ring_cap(P);
  const TmRing slot_of{rcap, (uint32_t)(0x100000000ull / rcap)};
  unsigned long long* key = (unsigned long long*)smem;
  uint16_t* ring = (uint16_t*)(smem + (size_t)P * 8);
  uint32_t* mark = (uint32_t*)(smem + (size_t)P * 8 + (size_t)rcap * 2);
  const uint32_t n_words = (P + 31) / 32;
  __shared__ uint32_t ctl[8];  // TAIL, ABORT
  constexpr int TAIL = 1, ABORT = 2;
  __shared__ unsigned long long hb;  // (head << 32) | busy
  __shared__ unsigned long long sink[64];
  __shared__ uint32_t s_cnt[TM_KMAX];                  // messages this member sent each target this superstep
  __shared__ uint32_t s_counts[TM_KMAX * TM_KMAX];     // the team's counts of this superstep
  __shared__ uint32_t s_team, s_mem, s_row, s_stop;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;

  if (tid == 0) {  // membership by arrival: only running workgroups form teams
    const uint32_t slot = atomicAdd(&a.rows_ctr[1], 1u);
    s_team = slot / K;
    s_mem = slot % K;
  }
  __syncthreads();
  const uint32_t team = s_team, mem = s_mem;
  if (team >= a.n_teams) return;
  uint32_t* tctl = a.team_ctl + (size_t)team * TM_CTL_WORDS;
  // tctl[0] row, [1] arrive, [2] abort, [4 + (p * K + s) * K + d] counts
  const uint32_t base = mem * P, Pm = min(P, a.n > base ? a.n - base : 0u);
  const __amdgpu_buffer_rsrc_t arcs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.team_arc, 0, (int)(a.n_arcs * 12u), 0x00020000);
  // the team's outbox: 2 parities x K sources x K targets x cap 16-byte messages
  const __amdgpu_buffer_rsrc_t box = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.outbox + (size_t)team * 2 * K * K * a.cap), 0, (int)(2 * K * K * a.cap * 16u), 0x00020000);
  uint32_t barrier_no = 0, parity = 0;
  unsigned long long n_rel = 0, n_msg = 0, n_steps = 0;
  // measurement only (a.work): thread 0's wall clock per part of the search: row claim,
  // setup and bounds, local phase, remote pass, exchange (barrier), apply, output
  unsigned long long t_part[7] = {}, t_last = a.work ? wall_clock64() : 0;
  auto tick = [&](int i) {
    if (a.work && tid == 0) {
      const unsigned long long t = wall_clock64();
      t_part[i] += t - t_last;
      t_last = t;
    }
  };
  uint32_t n_items = a.n_items, pbase = 0;
  if (a.plan_ctl) {
    pbase = a.plan_ctl[2 * a.plan_ph];
    n_items = a.plan_ctl[2 * a.plan_ph + 1];
  }
  __shared__ uint32_t s_ub[SSSP_KB_MAX][3];  // the row's usable bound rows: row, latency, exact
  __shared__ uint32_t s_nub;

  // team barrier: every member arrives once; waits for all K (budgeted: an abort ends the team)
  auto team_barrier = [&]() -> bool {
    barrier_no++;
    if (tid == 0) {
      uint32_t stop = 0;
      atomicAdd(&tctl[1], 1u);  // agent scope: the sc1 stores before it are drained (vmcnt(0) + barrier)
      const uint32_t target = barrier_no * K;
      uint32_t spins = 0;
      while (__hip_atomic_load(&tctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (__hip_atomic_load(&tctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          stop = 1;
          break;
        }
        if (++spins > a.spin_max) {
          __hip_atomic_store(&tctl[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          stop = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      s_stop = stop;
    }
    __syncthreads();
    return s_stop == 0;
  };
  auto drain = []() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };

  for (;;) {
    // ---- the row: claimed by member 0, published through the team's control block
    if (mem == 0 && tid == 0) {
      const uint32_t i = atomicAdd(&a.rows_ctr[0], 1u);
      __hip_atomic_store(&tctl[0], i < n_items ? i : TM_ROW_END, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    drain();
    __syncthreads();
    if (!team_barrier()) return;
    if (tid == 0) s_row = __hip_atomic_load(&tctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    tick(0);
    if (s_row == TM_ROW_END) break;
    const uint32_t item = s_row;
    const uint32_t row = a.blk_rows ? a.blk_rows[pbase + item] : a.row_begin + item;
    const uint32_t src = a.used[row];
    // ---- setup: keys, queue, marks
    for (uint32_t v = tid; v < P; v += NT) key[v] = TM_INF;
    for (uint32_t i = tid; i < rcap; i += NT) ring[i] = TM_EMPTY;
    for (uint32_t w = tid; w < n_words; w += NT) mark[w] = 0;
    if (tid < 8) ctl[tid] = 0;
    if (tid < TM_KMAX) s_cnt[tid] = 0;
    if (tid == 0) hb = 0;
    if (a.ub_row && tid < 64) {  // (sg_sssp.hip: a row that gave up gives no bounds, a saturated one bounds only)
      const size_t at = (size_t)(pbase + item) * SSSP_KB_MAX;
      const uint32_t e = tid < SSSP_KB_MAX ? a.ub_row[at + tid] : ~0u;
      const uint32_t w = tid < SSSP_KB_MAX ? a.ub_w[at + tid] : 0u;
      const uint32_t srow = e & ~SSSP_UB_EXACT;
      const uint32_t sf = e != ~0u ? a.sat_row[srow - a.row_begin] : 2u;
      const bool on = sf != 2u;
      const uint64_t mk = __ballot(on);
      if (on) {
        const int at2 = __popcll(mk & ((1ull << tid) - 1));
        s_ub[at2][0] = srow;
        s_ub[at2][1] = w;
        s_ub[at2][2] = (e & SSSP_UB_EXACT) && sf == 0u;
      }
      if (tid == 0) s_nub = (uint32_t)__popcll(mk);
    }
    __syncthreads();
    if (a.ub_row && s_nub) {
      // Bounds and exact seeds (sg_sssp.hip "Bounds", "Exact seeds") for this member's
      // columns: the bound rows are final (an earlier phase's launch)
      const int nb = (int)s_nub;
      constexpr uint32_t OOB = 0x80000000u;
      const uint32_t* mj = a.mem_used + (size_t)mem * a.n_used;
      const uint32_t n_mine = a.mem_n[mem];
      for (uint32_t i = tid; i < n_mine; i += NT) {
        const uint32_t j = mj[i], vj = a.used[j];
        const bool own = true;
        uint64_t m = ~0ull, ex = ~0ull;
        for (int k = 0; k < nb; k++) {
          const uint32_t sr = s_ub[k][0], w = s_ub[k][1];
          const bool exact = s_ub[k][2];
          const size_t rb = (size_t)(sr - a.row_begin) * a.n_used;
          const __amdgpu_buffer_rsrc_t rl =
              __builtin_amdgcn_make_buffer_rsrc((void*)(a.out_lat + rb), 0, (int)(a.n_used * 8u), 0x00020000);
          const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(
              (void*)(a.out_loss + rb), 0, (int)(exact ? a.n_used * 4u : 0u), 0x00020000);
          const auto x = __builtin_amdgcn_raw_buffer_load_b64(rl, own ? j * 8u : OOB, 0, 0);
          const uint32_t f = __builtin_amdgcn_raw_buffer_load_b32(rf, own ? j * 4u : OOB, 0, 0);
          const uint64_t ub = (((uint64_t)x[1] << 32) | x[0]) + w;  // w < 2^32: a wrap means >= 2^64
          if (!own || ub < w) continue;
          m = min(m, ub);
          if (exact && ub < LAT32_SAT && j != sr) ex = min(ex, (ub << 32) | ((uint64_t)f << 1));
        }
        uint64_t kv = m < LAT32_SAT - 1 ? ((m + 1) << 32) | ((uint64_t)0x3F800000u << 1) : TM_INF;
        kv = min(kv, ex);
        if (kv != TM_INF) key[vj - base] = kv;
      }
      __syncthreads();
    }
    if (tid == 0 && src - base < Pm) {
      key[src - base] = 1ull;  // PathProperties::default(), dirty and queued
      ring[0] = (uint16_t)(src - base);
      ctl[TAIL] = 1;
    }
    // every member set up before any message of this row is applied
    drain();
    __syncthreads();
    if (!team_barrier()) goto aborted;
    tick(1);
    for (;;) {  // supersteps
      // ---- 1. local phase (sg_sssp.hip's queue; arcs to own nodes only)
      {
        uint32_t spins = 0;
        for (;;) {
          uint32_t h = 0, k = 0;
          if (lane == 0) {
            for (;;) {
              const unsigned long long w = __hip_atomic_load(&hb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              const uint32_t hh = (uint32_t)(w >> 32),
                             t = __hip_atomic_load(&ctl[TAIL], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              if (t == hh) break;
              const uint32_t kk = min(64u, t - hh);
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
          if (__builtin_amdgcn_readfirstlane(
                  __hip_atomic_load(&ctl[ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
            break;
          if (!k) {
            uint32_t q = 0;
            if (lane == 0) {
              const unsigned long long w = __hip_atomic_load(&hb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              __atomic_signal_fence(__ATOMIC_SEQ_CST);
              q = (w & 0xFFFFFFFFull) == 0 &&
                  (uint32_t)(w >> 32) == __hip_atomic_load(&ctl[TAIL], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (__builtin_amdgcn_readfirstlane(q)) break;  // quiescent
            if (++spins > a.spin_max) {
              if (lane == 0) atomicExch(&ctl[ABORT], 1u);
              break;
            }
            __builtin_amdgcn_s_sleep(2);
            continue;
          }
          // pop the claimed entries
          const bool on = lane < (int)k;
          uint32_t u = 0, a0 = 0, a1 = 0, am = 0;
          uint64_t ku = 0;
          bool stuck = false;
          if (on) {
            volatile uint16_t* slot = &ring[slot_of(h + lane)];
            uint16_t x;
            uint32_t sp = 0;
            while ((x = *slot) == TM_EMPTY && ++sp < a.spin_max) __builtin_amdgcn_s_sleep(0);
            stuck = x == TM_EMPTY;
            *slot = TM_EMPTY;
            u = stuck ? 0 : x;
            const uint32_t ug = base + u;
            a0 = a.out_off[ug];
            a1 = a.out_off[ug + 1];
            am = a.team_mid[ug];
            ku = __hip_atomic_fetch_and(&key[u], ~1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & ~1ull;
            if (a1 - a0 > am) atomicOr(&mark[u >> 5], 1u << (u & 31));  // its remote arcs: the remote pass
          }
          if (__any(stuck)) {
            if (lane == 0) atomicExch(&ctl[ABORT], 1u);
            break;
          }
          const uint32_t deg = on ? am : 0u;
          const uint32_t dmax = __builtin_amdgcn_readlane(wave_incl_max(deg), 63);
          if (a.work) n_rel += __builtin_amdgcn_readlane(wave_incl_sum(deg), 63);
          for (uint32_t j0 = 0; j0 < dmax; j0 += TM_LA) {
            uint32_t v[TM_LA], lat[TM_LA], om[TM_LA];
            bool valid[TM_LA];
#pragma unroll
            for (int c = 0; c < TM_LA; c++) {
              valid[c] = j0 + c < deg;
              const auto r = __builtin_amdgcn_raw_buffer_load_b96(arcs, valid[c] ? (a0 + j0 + c) * 12u : 0x80000000u,
                                                                  0, 0);
              v[c] = r[0] - base;
              lat[c] = r[1];
              om[c] = r[2];
            }
            uint64_t cd[TM_LA], old[TM_LA];
#pragma unroll
            for (int c = 0; c < TM_LA; c++) {
              const uint64_t cand = tk_relax(ku, lat[c], __uint_as_float(om[c]));
              const bool ok = valid[c] && tk_lat(cand) != LAT32_SAT;
              cd[c] = ok ? cand : ~0ull;
              old[c] = __hip_atomic_fetch_min(ok ? &key[v[c]] : &sink[lane], (unsigned long long)cd[c],
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t lt = (1ull << lane) - 1;
            uint64_t mq[TM_LA];
            bool app[TM_LA];
            uint32_t tot = 0;
#pragma unroll
            for (int c = 0; c < TM_LA; c++) {
              app[c] = (old[c] >> 1) > (cd[c] >> 1) && !(old[c] & 1ull);
              mq[c] = __ballot(app[c]);
              tot += (uint32_t)__popcll(mq[c]);
            }
            if (tot) {
              uint32_t b = 0;
              if (lane == 0) b = atomicAdd(&ctl[TAIL], tot);
              b = __builtin_amdgcn_readfirstlane(b);
#pragma unroll
              for (int c = 0; c < TM_LA; c++) {
                if (app[c]) ring[slot_of(b + (uint32_t)__popcll(mq[c] & lt))] = (uint16_t)v[c];
                b += (uint32_t)__popcll(mq[c]);
              }
            }
          }
          if (lane == 0) atomicSub(&hb, 1ull);  // release the claim after this wave's appends
        }
      }
      __syncthreads();
      tick(2);
      if (ctl[ABORT]) goto aborted;
      // ---- 2. remote pass: every marked node relaxes its arcs to other members once
      {
        // the marked nodes into the (empty) queue: lane l takes bitmap word w0 + l, bit by bit
        for (uint32_t w0 = wv * 64; w0 < n_words; w0 += NT) {
          const uint32_t w = w0 + lane;
          uint32_t bits = w < n_words ? mark[w] : 0u;
          if (w < n_words) mark[w] = 0;
          for (;;) {
            const bool has = bits != 0;
            if (!__any(has)) break;
            const uint32_t u = w * 32 + (has ? (uint32_t)__builtin_ctz(bits) : 0u);
            if (has) bits &= bits - 1;
            const uint64_t m = __ballot(has);
            uint32_t b = 0;
            if (lane == 0) b = atomicAdd(&ctl[TAIL], (uint32_t)__popcll(m));
            b = __builtin_amdgcn_readfirstlane(b);
            if (has) ring[slot_of(b + (uint32_t)__popcll(m & ((1ull << lane) - 1)))] = (uint16_t)u;
          }
        }
        __syncthreads();
        const uint32_t head0 = (uint32_t)(hb >> 32), tail0 = ctl[TAIL];
        __syncthreads();
        // claimed 64 at a time from a workgroup counter (nothing is appended in this pass)
        __shared__ uint32_t s_claim;
        if (tid == 0) s_claim = head0;
        __syncthreads();
        for (;;) {
          uint32_t h = 0;
          if (lane == 0) h = atomicAdd(&s_claim, 64u);
          h = __builtin_amdgcn_readfirstlane(h);
          if (h >= tail0) break;
          const bool on = h + lane < tail0;
          uint32_t u = 0, a0 = 0, a1 = 0;
          uint64_t ku = 0;
          if (on) {
            const uint32_t sl = slot_of(h + lane);
            u = ring[sl];
            ring[sl] = TM_EMPTY;
            const uint32_t ug = base + u;
            a1 = a.out_off[ug + 1];
            a0 = a.out_off[ug] + a.team_mid[ug];
            ku = key[u] & ~1ull;
          }
          const uint32_t deg = on ? a1 - a0 : 0u;
          const uint32_t dmax = __builtin_amdgcn_readlane(wave_incl_max(deg), 63);
          if (a.work) n_rel += __builtin_amdgcn_readlane(wave_incl_sum(deg), 63);
          for (uint32_t j0 = 0; j0 < dmax; j0 += TM_LA) {
            uint32_t tv[TM_LA], td[TM_LA], pos[TM_LA];
            uint64_t cd[TM_LA];
            bool ok[TM_LA];
#pragma unroll
            for (int c = 0; c < TM_LA; c++) {
              const bool valid = j0 + c < deg;
              const auto r = __builtin_amdgcn_raw_buffer_load_b96(arcs, valid ? (a0 + j0 + c) * 12u : 0x80000000u, 0,
                                                                  0);
              cd[c] = tk_relax(ku, r[1], __uint_as_float(r[2]));
              ok[c] = valid && tk_lat(cd[c]) != LAT32_SAT;
              td[c] = r[0] / P;
              tv[c] = r[0] - td[c] * P;
              pos[c] = 0;
            }
            // slots: one LDS add per target member and wave (64 lanes adding to one
            // LDS word would serialise), then each message's rank among the wave's
            const uint64_t lt = (1ull << lane) - 1;
            for (uint32_t d = 0; d < K; d++) {
              uint64_t mk[TM_LA];
              uint32_t tot = 0;
#pragma unroll
              for (int c = 0; c < TM_LA; c++) {
                mk[c] = __ballot(ok[c] && td[c] == d);
                tot += (uint32_t)__popcll(mk[c]);
              }
              if (!tot) continue;
              uint32_t b = 0;
              if (lane == 0) b = atomicAdd(&s_cnt[d], tot);
              b = __builtin_amdgcn_readfirstlane(b);
#pragma unroll
              for (int c = 0; c < TM_LA; c++) {
                if (ok[c] && td[c] == d) pos[c] = b + (uint32_t)__popcll(mk[c] & lt);
                b += (uint32_t)__popcll(mk[c]);
              }
            }
#pragma unroll
            for (int c = 0; c < TM_LA; c++) {
              if (!ok[c]) continue;
              if (pos[c] < a.cap) {  // (a block holds every arc between two members: never full)
                const uint32_t at = ((parity * K + mem) * K + td[c]) * a.cap + pos[c];
                const v4u msg = {tv[c], (uint32_t)cd[c], (uint32_t)(cd[c] >> 32), 0u};
                __builtin_amdgcn_raw_buffer_store_b128(msg, box, at * 16u, 0, TM_SC1);  // write-through
              } else {
                atomicExch(&ctl[ABORT], 1u);
              }
            }
          }
        }
        if (tid == 0) {  // the queue is empty again
          hb = (unsigned long long)tail0 << 32;
        }
      }
      // ---- 3. exchange: counts published behind every wave's drained stores
      drain();
      __syncthreads();
      tick(3);
      if (ctl[ABORT]) goto aborted;
      if (tid < (int)K)
        __hip_atomic_store(&tctl[4 + (parity * K + mem) * K + tid], s_cnt[tid], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      if (a.work && tid == 0)
        for (uint32_t d = 0; d < K; d++) n_msg += s_cnt[d];
      drain();
      __syncthreads();
      if (!team_barrier()) goto aborted;
      if (tid < (int)(K * K))
        s_counts[tid] = __hip_atomic_load(&tctl[4 + parity * K * K + tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tid < TM_KMAX) s_cnt[tid] = 0;
      __syncthreads();
      tick(4);
      uint32_t total = 0;
      for (uint32_t i = 0; i < K * K; i++) total += s_counts[i];
      n_steps++;
      if (total == 0) break;  // nobody sent anything: the row is final (every member reads the same counts)
      // ---- 4. apply the messages addressed to this member
      for (uint32_t s = 0; s < K; s++) {
        if (s == mem) continue;
        const uint32_t c = min(s_counts[s * K + mem], a.cap);
        const uint32_t blk = ((parity * K + s) * K + mem) * a.cap;
        for (uint32_t i0 = wv * 64; i0 < c; i0 += NT) {
          const uint32_t i = i0 + lane;
          const bool on = i < c;
          uint32_t v = 0;
          uint64_t cd = ~0ull, old = ~0ull;
          if (on) {
            const v4u msg = __builtin_amdgcn_raw_buffer_load_b128(box, (blk + i) * 16u, 0, TM_SC1);
            v = msg[0];
            cd = ((uint64_t)msg[2] << 32) | msg[1];
            old = __hip_atomic_fetch_min(&key[v], (unsigned long long)cd, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          const bool app = on && (old >> 1) > (cd >> 1) && !(old & 1ull);
          const uint64_t m = __ballot(app);
          if (m) {
            uint32_t b = 0;
            if (lane == 0) b = atomicAdd(&ctl[TAIL], (uint32_t)__popcll(m));
            b = __builtin_amdgcn_readfirstlane(b);
            if (app) ring[slot_of(b + (uint32_t)__popcll(m & ((1ull << lane) - 1)))] = (uint16_t)v;
          }
        }
      }
      parity ^= 1u;
      __syncthreads();
      tick(5);
    }
    // ---- the member's columns of the row (diagonal = the raw self-loop, graph/mod.rs:210-217)
    {
      const size_t orow = (size_t)(row - a.row_begin) * a.n_used;
      bool sat = false;
      const uint32_t* mj = a.mem_used + (size_t)mem * a.n_used;
      const uint32_t n_mine = a.mem_n[mem];
      for (uint32_t i = tid; i < n_mine; i += NT) {
        const uint32_t j = mj[i], vj = a.used[j];
        uint64_t l;
        float f;
        if (j == row) {
          const uint32_t e = a.self_edge[vj];
          l = a.e_lat[e];
          f = a.e_loss[e];
        } else {
          const uint64_t kk = key[vj - base];
          sat |= tk_lat(kk) == LAT32_SAT;
          l = tk_lat(kk);
          f = __uint_as_float(tk_loss_bits(kk));
        }
        __builtin_nontemporal_store(l, &a.out_lat[orow + j]);
        __builtin_nontemporal_store(f, &a.out_loss[orow + j]);
      }
      if (__any(sat) && lane == 0) a.sat_row[row - a.row_begin] = 1u;
    }
    tick(6);
    parity ^= 1u;  // (keeps every member's parity in step: the loop above left by `break` before flipping)
    __syncthreads();
    continue;
  aborted:
    // flag the row for the wide kernel; the team stops (the host flags the rows nobody claimed)
    if (tid == 0) {
      a.sat_row[row - a.row_begin] = 2u;
      __hip_atomic_store(&tctl[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    break;
  }
  if (a.work && lane == 0) {  // (n_rel is wave-uniform; n_msg is thread 0's)
    if (n_rel) atomicAdd(&a.work[0], n_rel);
    if (n_msg) atomicAdd(&a.work[1], n_msg);
    if (tid == 0 && mem == 0 && n_steps) atomicAdd(&a.work[2], n_steps);
    if (tid == 0)
      for (int i = 0; i < 7; i++) atomicAdd(&a.work[3 + i], t_part[i]);
  }
}

}  // namespace

bool sssp_team_fits(uint32_t n, uint32_t K) {
  if (K < 2 || K > (uint32_t)TM_KMAX) return false;
  const uint32_t P = (n + K - 1) / K;
  return P < TM_EMPTY && tm_lds_bytes(P) + TM_STATIC_LDS <= TM_LDS;
}

uint32_t sssp_team_size(uint32_t n) {
  for (uint32_t K = 2; K <= (uint32_t)TM_KMAX; K++)
    if (sssp_team_fits(n, K)) return K;
  return 0;
}

// The team's arc order and the outbox blocks' capacity (the largest (member,
// member) arc count): once per build (one synchronisation).
uint32_t sssp_team_prepare(sg_ctx* ctx, sg_net* net, uint32_t K) {
  hipStream_t st = ctx->stream;
  const uint32_t n = net->n_nodes;
  if (!sssp_team_fits(n, K)) throw Error(SG_ERR_INVALID_ARG, "graph too large for the team search");
  if ((uint64_t)net->n_arcs * 12 >= (1ull << 31)) throw Error(SG_ERR_INVALID_ARG, "too many arcs for 32-bit offsets");
  const uint32_t P = (n + K - 1) / K;
  uint32_t* team_arc = ctx->r_team_arc.get<uint32_t>(3 * (size_t)std::max(net->n_arcs, 1u));
  uint32_t* team_mid = ctx->r_team_mid.get<uint32_t>(n);
  uint32_t* pair = ctx->r_team_pair.get<uint32_t>(TM_KMAX * TM_KMAX);
  SG_HIP(hipMemsetAsync(pair, 0, TM_KMAX * TM_KMAX * 4, st));
  hipLaunchKernelGGL(k_team_arcs, dim3(grid_for(n, 256)), dim3(256), 0, st, net->out_off, net->out_arc, n, P, K,
                     team_arc, team_mid, pair);
  SG_CHECK_LAUNCH();
  std::vector<uint32_t> hp(K * K);
  copy_to_host(ctx, hp.data(), pair, K * K * 4);
  uint32_t cap = 64;
  for (uint32_t i = 0; i < K * K; i++) cap = std::max(cap, hp[i]);
  return cap;
}

namespace {
// Per member m, the used indices j with used[j] in m's nodes, ascending: the
// member's columns of a row (bounds in, table out) without a scan of every j.
__global__ void __launch_bounds__(1024) k_team_used(const uint32_t* __restrict__ used, uint32_t n_used, uint32_t P,
                                                    uint32_t* __restrict__ mem_used, uint32_t* __restrict__ mem_n) {
  __shared__ uint32_t wsum[16], s_base;
  const uint32_t m = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) s_base = 0;
  __syncthreads();
  for (uint32_t j0 = 0; j0 < n_used; j0 += 1024) {
    const uint32_t j = j0 + tid;
    const bool mine = j < n_used && used[j] / P == m;
    const uint64_t mk = __ballot(mine);
    if (lane == 0) wsum[wv] = (uint32_t)__popcll(mk);
    __syncthreads();
    uint32_t off = s_base;
    for (int w = 0; w < wv; w++) off += wsum[w];
    if (mine) mem_used[(size_t)m * n_used + off + (uint32_t)__popcll(mk & ((1ull << lane) - 1))] = j;
    __syncthreads();
    if (tid == 0)
      for (int w = 0; w < 16; w++) s_base += wsum[w];
    __syncthreads();
  }
  if (tid == 0) mem_n[m] = s_base;
}

// items a launch's teams never claimed (every team gave up) go to the wide kernel
__global__ void k_team_unclaimed(const uint32_t* __restrict__ rows_ctr, uint32_t n_items,
                                 const uint32_t* __restrict__ plan_ctl, int ph, const uint32_t* __restrict__ blk_rows,
                                 uint32_t row_begin, uint32_t* __restrict__ sat_row) {
  uint32_t pbase = 0;
  if (plan_ctl) {
    pbase = plan_ctl[2 * ph];
    n_items = plan_ctl[2 * ph + 1];
  }
  for (uint32_t i = rows_ctr[0] + blockIdx.x * blockDim.x + threadIdx.x; i < n_items; i += gridDim.x * blockDim.x)
    sat_row[(blk_rows ? blk_rows[pbase + i] : row_begin + i) - row_begin] = 2u;
}
}  // namespace

// Rows [row_begin, row_end) of the table (or, with a plan, phase ph's rows) with
// teams of K workgroups; sat_row (device, zeroed by the caller) gets 1 for rows to
// redo wide (saturated) and 2 for rows a team gave up on or never claimed.
void launch_sssp_team(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used, uint32_t row_begin,
                      uint32_t row_end, uint64_t* out_lat, float* out_loss, uint32_t* sat_row, uint32_t K,
                      uint32_t cap, unsigned long long* work, const SsspDevPlan* plan, int ph) {
  hipStream_t st = ctx->stream;
  const uint32_t n = net->n_nodes, rows = row_end - row_begin;
  const uint32_t P = (n + K - 1) / K;
  const uint32_t n_teams = std::max(1u, (uint32_t)ctx->n_cu / K);
  const size_t box = (size_t)n_teams * 2 * K * K * cap;
  if ((size_t)2 * K * K * cap * 16 >= (1ull << 31)) throw Error(SG_ERR_INVALID_ARG, "team outbox too large");
  uint4* outbox = ctx->r_team_box.get<uint4>(box);
  uint32_t* tctl = ctx->r_team_ctl.get<uint32_t>((size_t)n_teams * TM_CTL_WORDS + 2);
  uint32_t* rows_ctr = tctl + (size_t)n_teams * TM_CTL_WORDS;
  SG_HIP(hipMemsetAsync(tctl, 0, ((size_t)n_teams * TM_CTL_WORDS + 2) * 4, st));
  const char* sm = getenv("SG_SSSP_SPIN_MAX");
  TeamArgs ta;
  ta.out_off = net->out_off;
  ta.team_arc = ctx->r_team_arc.get<uint32_t>(3 * (size_t)std::max(net->n_arcs, 1u));
  ta.team_mid = ctx->r_team_mid.get<uint32_t>(n);
  ta.n = n;
  ta.n_arcs = net->n_arcs;
  ta.P = P;
  ta.K = K;
  ta.used = d_used;
  ta.n_used = n_used;
  uint32_t* mem_used = ctx->r_team_used.get<uint32_t>((size_t)K * n_used + K);
  ta.mem_used = mem_used;
  ta.mem_n = mem_used + (size_t)K * n_used;
  if (!plan || ph == 0)  // (the later phases of a plan reuse the lists)
    hipLaunchKernelGGL(k_team_used, dim3(K), dim3(1024), 0, st, d_used, n_used, P, mem_used,
                       mem_used + (size_t)K * n_used);
  ta.row_begin = row_begin;
  ta.self_edge = net->self_edge;
  ta.e_lat = net->e_lat;
  ta.e_loss = net->e_loss;
  ta.out_lat = out_lat;
  ta.out_loss = out_loss;
  ta.sat_row = sat_row;
  ta.rows_ctr = rows_ctr;
  ta.n_items = rows;
  ta.n_teams = n_teams;
  ta.team_ctl = tctl;
  ta.outbox = outbox;
  ta.cap = cap;
  ta.spin_max = sm && *sm ? (uint32_t)std::max(1, atoi(sm)) : (1u << 22);
  ta.work = work;
  ta.blk_rows = plan ? plan->list : nullptr;
  ta.ub_row = plan && ph > 0 ? plan->ub_row : nullptr;
  ta.ub_w = plan && ph > 0 ? plan->ub_w : nullptr;
  ta.plan_ctl = plan ? plan->ctl : nullptr;
  ta.plan_ph = ph;
  const size_t lds = tm_lds_bytes(P);
  SG_HIP(hipFuncSetAttribute((const void*)k_sssp_team, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)(TM_LDS - TM_STATIC_LDS)));
  {
    TimedLaunch tl(ctx, ph > 0 ? "sssp_team_bounded" : "sssp_team", 0.0);
    hipLaunchKernelGGL(k_sssp_team, dim3(n_teams * K), dim3(TM_THREADS), lds, st, ta);
  }
  hipLaunchKernelGGL(k_team_unclaimed, dim3(grid_for(rows, 256, 64)), dim3(256), 0, st, rows_ctr, rows,
                     plan ? plan->ctl : nullptr, ph, plan ? plan->list : nullptr, row_begin, sat_row);
  SG_CHECK_LAUNCH();
}

}  // namespace sg
