// sg_bucket.hip -- per-source shortest paths on sparse graphs past the LDS (C5: 50k nodes).
//
// Replaces, for sparse graphs whose distance row no longer fits a CU's LDS, the
// per-source petgraph::algo::dijkstra of NetworkGraph::compute_shortest_paths
// (graph/mod.rs:190-208).  sg_sssp.hip keeps a whole row of 8-B keys in LDS, which
// stops at ~10.9k nodes; the batched-source slab (sg_routing.hip k_relax_w2) goes
// on past it but re-gathers a row whenever any of its 64 sources improved it:
// 10.5x Dijkstra's relaxations at C5.  This search does Dijkstra's work at any
// size by keeping in LDS only what one distance band needs.
//
// Delta-stepping with a ring of buckets.  Bucket k holds the candidate keys whose
// latency lies in [k Delta, (k + 1) Delta) (Delta: the smallest arc latency by default, so
// that a band never relaxes into itself).  Buckets are
// processed in order; processing bucket b:
//   A. its entries are read from global memory and offered to an LDS hash table
//      that holds the band's keys (node -> flagged key, the 64-bit atomic min of
//      sg_sssp.hip); a node already settled is skipped;
//   B. the hash's dirty nodes are relaxed through the asynchronous LDS queue of
//      sg_sssp.hip until quiescent.  A candidate that lands in bucket b goes to
//      the hash (and is relaxed again if it improved); one that lands in a later
//      bucket k < b + R is appended to ring slot k mod R; beyond that, to a far
//      list; a candidate to a settled node is dropped;
//   C. every node of the hash is settled: its key is final, stored to the
//      workgroup's scratch row, and its bit set in an LDS bitmap.
// Exactness.  Edge latency >= 1 ns (graph/mod.rs:105-107) and the f32 loss fold
// is monotone, so a node's PathProperties-minimal path (graph/mod.rs:297-313)
// reaches it from a predecessor of strictly smaller latency.  By induction over
// the buckets, when bucket b starts every node of smaller latency is settled with
// its final key and has been relaxed (A/B of its own bucket), so the final key of
// every node in bucket b is offered there -- as an entry appended when its
// predecessor was relaxed, or inside the band by B's fixed point (sg_sssp.hip's
// proof: any relaxation order reaches it).  Keys are compared as the packed
// (latency, loss) of sg_sssp.hip, the fold applies the edge on the right
// (sg_device.h fold_loss), so the settled key is petgraph's.  A candidate whose
// latency saturates (LAT32_SAT) is never offered: its node stays unsettled, and
// an unsettled node flags the row for the wide kernel (sg_routing.hip run_wide),
// as unreachable nodes do.
//
// Memory.  LDS holds the band: the hash (HS slots of node id + flagged key), the
// queue of hash slots, the settled bitmap (n bits), and per ring slot a table of
// the chunks that hold its entries.  Entries are 12-B records {node, latency,
// bits(loss)} in 256-entry chunks of a per-workgroup arena in HBM (chunks of a
// processed bucket return to an LDS free stack, so the arena holds only the
// entries in flight and stays in L2 / the Infinity Cache).  An entry is written
// once and read once; at C5 a row appends ~200k entries (0.5 per arc), against the
// slab's ~10 full-row gathers per source.
//
// Safety valves (never reached by a correct search of a graph the host sized the
// workspace for): a hash that fills, a bucket past BK_MAXCH chunks, an arena
// without a free chunk, a spin budget.  The wave that hits one flags the row for
// the wide kernel and the whole workgroup leaves (sg_sssp.hip give_up).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "sg_device.h"
#include "sg_internal.h"

namespace sg {

constexpr uint32_t BK_R = 128;             // ring slots (buckets in flight), at most
constexpr uint32_t BK_SLOTS = BK_R + 2;    // + two far lists (the current one and the one being filled)
constexpr uint32_t BK_CH_LOG = 8;
constexpr uint32_t BK_CH = 1u << BK_CH_LOG;  // entries per chunk
constexpr uint32_t BK_MAXCH = 32;          // chunks per bucket: 8,192 entries
constexpr uint16_t CH_EMPTY = 0xFFFF;
constexpr uint32_t HID_EMPTY = 0xFFFFFFFFu;
constexpr uint16_t QB_EMPTY = 0xFFFF;
constexpr int BK_SC1 = 16;  // buffer cache-policy bits: sc1 (L2-served, past this CU's L1)

constexpr uint64_t BKEY_INF = ((uint64_t)LAT32_SAT << 32) | ((uint64_t)0x3F800000u << 1);  // (SAT, 1.0), clean
__device__ __forceinline__ uint32_t bkey_lat(uint64_t k) { return (uint32_t)(k >> 32); }
__device__ __forceinline__ uint32_t bkey_loss_bits(uint64_t k) { return ((uint32_t)k >> 1) & 0x7FFFFFFFu; }
__device__ __forceinline__ uint64_t bkey_relax(uint64_t ku, uint32_t edge_lat, float edge_om) {
  const uint32_t lat = __builtin_elementwise_add_sat(bkey_lat(ku), edge_lat);
  const float loss = fold_loss(__uint_as_float(bkey_loss_bits(ku)), edge_om);
  return ((uint64_t)lat << 32) | ((uint64_t)__float_as_uint(loss) << 1) | 1ull;
}

struct BkArgs {
  const uint32_t* out_off;
  const uint32_t* out_arc;
  uint32_t n, n_arcs;
  const uint32_t* used;
  uint32_t n_used, row_begin, rows;
  const uint32_t* self_edge;
  const uint64_t* e_lat;
  const float* e_loss;
  uint64_t* out_lat;
  float* out_loss;
  uint32_t* sat_row;
  uint32_t delta, dmul, ring, hs_log2, nch, stg_cap;  // dmul = floor((2^32 - 1) / delta)
  uint32_t* arena;                // nch * BK_CH entries of 3 u32 per workgroup
  unsigned long long* scratch;    // n keys per workgroup
  uint32_t* item_ctr;             // [claims, workgroups given up] (zeroed)
  uint32_t spin_max;
  int vec_out;
  uint32_t arena_words, scr_stride;  // k_sssp_band: u32 per workgroup's arena, keys per scratch row
  // k_sssp_band on the degree-class numbering (see k_band_classes): node ids of the used list in
  // it (the search, the settled bitmap and the scratch row use them; `used` stays the graph's for
  // the diagonal), the class table [first id x 17, first arc x 17] and the class-16 arc offsets
  const uint32_t* used_key;
  const uint32_t* cls;
  const uint32_t* hi_off;
  uint32_t npw;  // k_sssp_band: band nodes a wave settles per step (<= 64)
  // k_sssp_band's per-node append filter (null: off): per workgroup filt_stride bytes, one per node
  // (degree-class id): 0, or 1 + (the bucket of the best candidate appended for it so far mod 255)
  uint8_t* filt;
  uint32_t filt_stride;
  unsigned long long* work;       // COUNT: relaxations
  unsigned long long* diag;       // COUNT: [buckets, entries appended, far steps, pops] summed
};

// queue of hash slots: a power of two >= HS + 64 NW (each slot is queued at most once while dirty,
// and at most NW waves x 64 claimed entries are still being read; sg_sssp.hip sssp_ring_cap)
__host__ __device__ inline uint32_t bk_qcap(uint32_t hs, uint32_t nw) {
  uint32_t q = 64;
  while (q < hs + 64 * nw) q <<= 1;
  return q;
}
// lat / delta by a multiply-high and at most two corrections
__device__ __forceinline__ uint32_t bk_bucket(uint32_t lat, uint32_t delta, uint32_t dmul) {
  uint32_t q = __umulhi(lat, dmul);
  uint32_t r = lat - q * delta;
  if (r >= delta) {
    q++;
    r -= delta;
  }
  return r >= delta ? q + 1 : q;
}
// dynamic LDS: hid[HS] u32, hkey[HS] u64, ulist[HS] u16 (the slots in use), queue[qcap] u16,
// settled[nbw] u32, tab[BK_SLOTS][BK_MAXCH] u16, cnt[BK_SLOTS] u32, fstack[nch] u16, stg[stg] 16 B
struct BkLds {
  size_t o_hkey, o_ul, o_q, o_set, o_tab, o_cnt, o_fst, o_stg, bytes;
  __host__ __device__ BkLds(uint32_t n, uint32_t hs, uint32_t nch, uint32_t stg, uint32_t nw) {
    o_hkey = (size_t)hs * 4;
    o_ul = o_hkey + (size_t)hs * 8;
    o_q = o_ul + (size_t)hs * 2;
    o_set = o_q + (size_t)bk_qcap(hs, nw) * 2;
    o_tab = o_set + ((size_t)(n + 31) / 32 * 4 + 7) / 8 * 8;
    o_cnt = o_tab + (size_t)BK_SLOTS * BK_MAXCH * 2;
    o_fst = o_cnt + (size_t)BK_SLOTS * 4;
    o_stg = (o_fst + (size_t)nch * 2 + 15) / 16 * 16;
    bytes = o_stg + (size_t)stg * 16;
  }
};
constexpr size_t BK_STATIC_LDS = 4 * 16 + 16 + 512 + 64;

template <bool COUNT, int NT, int LA>
__global__ void __launch_bounds__(NT) k_sssp_bucket(BkArgs a) {
  constexpr uint32_t NW = NT / 64;
  extern __shared__ __align__(16) unsigned char smem[];
  const uint32_t HS = 1u << a.hs_log2, hmask = HS - 1, qcap = bk_qcap(HS, NW);
  const uint32_t n = a.n, R = a.ring, rmask = R - 1;
  const BkLds L(n, HS, a.nch, a.stg_cap, NW);
  uint32_t* hid = (uint32_t*)smem;
  unsigned long long* hkey = (unsigned long long*)(smem + L.o_hkey);
  uint16_t* ulist = (uint16_t*)(smem + L.o_ul);
  uint16_t* qring = (uint16_t*)(smem + L.o_q);
  uint32_t* settled = (uint32_t*)(smem + L.o_set);
  uint16_t* tab = (uint16_t*)(smem + L.o_tab);
  uint32_t* cnt = (uint32_t*)(smem + L.o_cnt);
  uint16_t* fstack = (uint16_t*)(smem + L.o_fst);
  uint4* stg = (uint4*)(smem + L.o_stg);
  const uint32_t nbw = (n + 31) / 32;
  // ctl: TAIL (queue tail), ABORT, FTOP (free stack top, signed), FBUMP (fresh chunks), NEXT (the next
  // bucket, or a far step / done), FMIN (a far step's bucket), FARMIN + f (far list f's smallest
  // bucket), STG (staged entries), UCNT (hash slots in use)
  constexpr int TAIL = 1, ABORT = 2, FTOP = 3, FBUMP = 4, NEXT = 5, FMIN = 6, FARMIN = 7, STG = 9, UCNT = 10;
  __shared__ uint32_t ctl[16];
  __shared__ unsigned long long hb;  // (queue head << 32) | busy waves
  __shared__ uint32_t s_item;
  __shared__ unsigned long long sink[64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr uint32_t NEXT_DONE = 0xFFFFFFFFu, NEXT_FAR = 0xFFFFFFFEu;

  // one-time state: the hash, the chunk tables and counts are clean between rows (every
  // bucket is consumed before a row ends), the free stack persists across rows
  for (uint32_t i = tid; i < HS; i += NT) {
    hid[i] = HID_EMPTY;
    hkey[i] = BKEY_INF;
  }
  for (uint32_t i = tid; i < BK_SLOTS * BK_MAXCH; i += NT) tab[i] = CH_EMPTY;
  for (uint32_t i = tid; i < BK_SLOTS; i += NT) cnt[i] = 0;
  if (tid < 16) ctl[tid] = tid == FARMIN || tid == FARMIN + 1 ? 0xFFFFFFFFu : 0u;
  if (tid < 64) sink[tid] = ~0ull;
  const size_t ent0 = (size_t)blockIdx.x * a.nch * BK_CH * 3;  // this workgroup's arena (u32 index)
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)(a.arena + ent0), 0,
                                                                      (int)(a.nch * BK_CH * 12u), 0x00020000);
  unsigned long long* scr = a.scratch + (size_t)blockIdx.x * n;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)scr, 0, (int)(n * 8u), 0x00020000);
  const __amdgpu_buffer_rsrc_t arcs = __builtin_amdgcn_make_buffer_rsrc((void*)a.out_arc, 0, (int)(a.n_arcs * 12u),
                                                                        0x00020000);
  const __amdgpu_buffer_rsrc_t roff = __builtin_amdgcn_make_buffer_rsrc((void*)a.out_off, 0, (int)((n + 1) * 4u),
                                                                        0x00020000);
  if (tid == 0) s_item = atomicAdd(a.item_ctr, 1u);
  auto ld = [](uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
  auto is_settled = [&](uint32_t v) { return (settled[v >> 5] >> (v & 31)) & 1u; };
  uint32_t row = 0;
  // Giving up (a safety valve): flag the row for the wide kernel, abort the workgroup; the
  // last persistent workgroup to give up flags the rows none claimed (sg_sssp.hip give_up)
  auto give_up = [&]() {
    if (atomicExch(&ctl[ABORT], 1u) == 0u) {
      a.sat_row[row - a.row_begin] = 2u;
      __threadfence();
      if (atomicAdd(&a.item_ctr[1], 1u) == gridDim.x - 1) {
        const uint32_t c = __hip_atomic_load(&a.item_ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t i = min(c, a.rows); i < a.rows; i++) a.sat_row[i] = 2u;
      }
    }
  };
  unsigned long long n_rel = 0, n_app = 0, n_bk = 0, n_far = 0, n_pop = 0, n_claim = 0;
  unsigned long long cyc[4] = {0, 0, 0, 0};  // COUNT, thread 0: cycles in load + relax, settle, far steps, output
  unsigned long long t_mark = 0;
  // COUNT, per wave (lane 0): cycles in the load step, in claims (to the offsets, to the arcs, to the
  // appends, to the release), idle in the claim loop
  unsigned long long wc[6] = {0, 0, 0, 0, 0, 0};
  auto wclk = [&]() -> unsigned long long { return COUNT ? clock64() : 0ull; };
  auto stamp = [&](int k) {
    if (COUNT && tid == 0) {
      const unsigned long long t = clock64();
      if (k >= 0) cyc[k] += t - t_mark;
      t_mark = t;
    }
  };

  // The probe of node v's hash slot (inserting v if absent, and listing the slot); HS = a full
  // table (give up)
  auto hash_slot = [&](uint32_t v) -> uint32_t {
    uint32_t h = (v * 0x9E3779B1u) >> (32 - a.hs_log2);
    for (uint32_t p = 0; p < HS; p++) {
      const uint32_t id = ld(&hid[h]);
      if (id == v) return h;
      if (id == HID_EMPTY) {
        const uint32_t o = atomicCAS(&hid[h], HID_EMPTY, v);
        if (o == HID_EMPTY) {
          ulist[atomicAdd(&ctl[UCNT], 1u)] = (uint16_t)h;
          return h;
        }
        if (o == v) return h;
      }
      h = (h + 1) & hmask;
    }
    return HS;
  };
  // Queue the flagged lanes' hash slots: one tail add per call
  auto append_q = [&](bool app, uint32_t x) {
    const uint64_t m = __ballot(app);
    if (!m) return;
    uint32_t b0 = 0;
    if (lane == 0) b0 = atomicAdd(&ctl[TAIL], (uint32_t)__popcll(m));
    b0 = __builtin_amdgcn_readfirstlane(b0);
    if (app) qring[(b0 + (uint32_t)__popcll(m & ((1ull << lane) - 1))) & (qcap - 1)] = (uint16_t)x;
  };
  // Offer a flagged candidate to the band's hash; true: it improved a clean key (queue the slot)
  auto offer_hash = [&](bool on, uint32_t v, uint64_t cd, uint32_t& x) -> bool {
    x = on ? hash_slot(v) : HS;
    if (on && x == HS) give_up();
    const bool ok = on && x != HS;
    const uint64_t old = __hip_atomic_fetch_min(ok ? &hkey[x] : &sink[lane], (unsigned long long)(ok ? cd : ~0ull),
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return ok && (old >> 1) > (cd >> 1) && !(old & 1ull);
  };
  // A chunk for a bucket's next 256 entries: from the free stack, else fresh
  auto alloc_chunk = [&]() -> uint32_t {
    const int t = atomicSub((int*)&ctl[FTOP], 1) - 1;
    if (t >= 0) return fstack[t];
    const uint32_t id = atomicAdd(&ctl[FBUMP], 1u);
    if (id >= a.nch) {
      give_up();
      return 0u;
    }
    return id;
  };
  // Append entries (node, flagged key) to ring slots: NK per lane, slot s[c] (>= BK_SLOTS: none);
  // a far list keeps its smallest bucket.  The record goes to the LDS
  // staging array with its arena position (stored to the arena once the band is quiescent, so no
  // global store sits on a relaxation's dependent chain), or, `direct` or past the staging, straight
  // to the arena.  Must be called by whole waves (the staging claim is one add per wave and c).
  auto append_entries = [&](auto nk, const uint32_t* s, const uint32_t* v, const uint64_t* cd, bool direct) {
    constexpr int NK = decltype(nk)::value;
    uint32_t pos[NK];
#pragma unroll
    for (int c = 0; c < NK; c++)
      pos[c] = s[c] < BK_SLOTS ? atomicAdd(&cnt[s[c]], 1u) : 0u;
#pragma unroll
    for (int c = 0; c < NK; c++)
      if (s[c] >= BK_R && s[c] < BK_SLOTS)
        atomicMin(&ctl[FARMIN + (s[c] - BK_R)], bk_bucket(bkey_lat(cd[c]), a.delta, a.dmul));
#pragma unroll
    for (int c = 0; c < NK; c++) {
      if (s[c] < BK_SLOTS && (pos[c] >> BK_CH_LOG) < BK_MAXCH && (pos[c] & (BK_CH - 1)) == 0) {
        const uint32_t id = alloc_chunk();
        __hip_atomic_store(&tab[s[c] * BK_MAXCH + (pos[c] >> BK_CH_LOG)], (uint16_t)id, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    uint32_t sidx[NK];
    {  // staging positions: one add per call
      uint64_t m[NK];
      uint32_t tot = 0;
#pragma unroll
      for (int c = 0; c < NK; c++) {
        m[c] = __ballot(s[c] < BK_SLOTS);
        tot += (uint32_t)__popcll(m[c]);
      }
      uint32_t b0 = 0;
      if (!direct && tot && lane == 0) b0 = atomicAdd(&ctl[STG], tot);
      b0 = __builtin_amdgcn_readfirstlane(b0);
#pragma unroll
      for (int c = 0; c < NK; c++) {
        sidx[c] = b0 + (uint32_t)__popcll(m[c] & ((1ull << lane) - 1));
        b0 += (uint32_t)__popcll(m[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < NK; c++) {
      if (s[c] >= BK_SLOTS) continue;
      if ((pos[c] >> BK_CH_LOG) >= BK_MAXCH) {
        give_up();
        continue;
      }
      uint16_t* tp = &tab[s[c] * BK_MAXCH + (pos[c] >> BK_CH_LOG)];
      uint16_t id;
      uint32_t sp = 0;
      while ((id = __hip_atomic_load(tp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) == CH_EMPTY &&
             ++sp < a.spin_max)
        __builtin_amdgcn_s_sleep(0);
      if (id == CH_EMPTY) {
        give_up();
        continue;
      }
      const uint32_t e = ((uint32_t)id << BK_CH_LOG) | (pos[c] & (BK_CH - 1));
      if (!direct && sidx[c] < a.stg_cap) {
        stg[sidx[c]] = make_uint4(v[c], bkey_lat(cd[c]), bkey_loss_bits(cd[c]), e);
      } else {
        typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
        __builtin_amdgcn_raw_buffer_store_b96((u32x3){v[c], bkey_lat(cd[c]), bkey_loss_bits(cd[c])}, ra, e * 12u, 0,
                                              0);
      }
    }
    if (COUNT) {
#pragma unroll
      for (int c = 0; c < NK; c++) n_app += __popcll(__ballot(s[c] < BK_SLOTS));
    }
  };

  for (;;) {  // rows
    __syncthreads();  // s_item written (first row: above; later rows: in the previous row's output)
    const uint32_t bi = s_item;
    if (bi >= a.rows) break;
    row = a.row_begin + bi;
    const uint32_t src = a.used[row];
    for (uint32_t i = tid; i < nbw; i += NT) settled[i] = 0u;
    for (uint32_t i = tid; i < qcap; i += NT) qring[i] = QB_EMPTY;
    __syncthreads();
    if (tid == 0) {  // PathProperties::default() at the source, dirty and queued
      const uint32_t h = (src * 0x9E3779B1u) >> (32 - a.hs_log2);
      hid[h] = src;
      hkey[h] = 1ull;
      ulist[0] = (uint16_t)h;
      ctl[UCNT] = 1;
      ctl[STG] = 0;
      qring[0] = (uint16_t)h;
      ctl[TAIL] = 1;
      hb = NW;  // head 0, every wave busy with the first band's load (step A)
    }
    uint32_t b = 0;            // the bucket being processed
    uint32_t far = BK_R;       // the far list candidates past the ring go to
    __syncthreads();
    stamp(-1);
    for (;;) {  // buckets
      if (COUNT) n_bk++;
      const unsigned long long tA = wclk();
      // ---- A: bucket b's entries into the hash (its ring slot; a settled node's are stale).  Every
      // wave counts as busy until its part is offered, so the queue cannot look quiescent before.
      {
        const uint32_t sb = b & rmask, c = cnt[sb];
        constexpr int AG = 4;  // entries a lane loads at once
        for (uint32_t i0 = wv * 64; i0 < c; i0 += NT * AG) {  // whole waves (append_q is wave-wide)
          uint32_t v[AG];
          uint64_t cd[AG];
          bool on[AG];
#pragma unroll
          for (int g = 0; g < AG; g++) {
            const uint32_t i = i0 + g * NT + lane;
            on[g] = i < c;
            const uint32_t id = on[g] ? tab[sb * BK_MAXCH + (i >> BK_CH_LOG)] : 0u;
            const uint32_t e = (id << BK_CH_LOG) | (i & (BK_CH - 1));
            const auto r = __builtin_amdgcn_raw_buffer_load_b96(ra, on[g] ? e * 12u : 0x80000000u, 0, BK_SC1);
            v[g] = r[0];
            cd[g] = ((uint64_t)r[1] << 32) | ((uint64_t)r[2] << 1) | 1ull;
          }
#pragma unroll
          for (int g = 0; g < AG; g++) {
            const bool live = on[g] && !is_settled(v[g]);
            uint32_t x;
            const bool app = offer_hash(live, v[g], cd[g], x);
            append_q(app, x);
          }
        }
        if (lane == 0) atomicSub(&hb, 1ull);  // this wave's part is offered and queued
        if (COUNT) wc[0] += wclk() - tA;
      }
      // ---- B: relax the band's dirty nodes until the queue is quiescent
      uint32_t spins = 0;  // idle polls of this wave in this band (a safety valve)
      for (;;) {
        uint32_t h = 0, k = 0;
        if (lane == 0) {
          for (;;) {
            const unsigned long long w = __hip_atomic_load(&hb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t hh = (uint32_t)(w >> 32), t = ld(&ctl[TAIL]);
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
        if (COUNT && k && lane == 0) n_claim++;
        const unsigned long long t0 = wclk();
        if (__builtin_amdgcn_readfirstlane(ld(&ctl[ABORT]))) goto wave_exit;
        if (!k) {
          uint32_t q = 0;
          if (lane == 0) {
            const unsigned long long w = __hip_atomic_load(&hb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);  // (head, busy) before tail (sg_sssp.hip)
            q = (w & 0xFFFFFFFFull) == 0 && (uint32_t)(w >> 32) == ld(&ctl[TAIL]);
          }
          if (!__builtin_amdgcn_readfirstlane(q)) {
            if (++spins > a.spin_max) {
              if (lane == 0) give_up();
              goto wave_exit;
            }
            __builtin_amdgcn_s_sleep(1);
            if (COUNT) wc[5] += wclk() - t0;
            continue;
          }
          break;  // quiescent: every wave gets here
        }
        // pop the claimed hash slots (a slot claimed before its writer stored it reads EMPTY)
        const bool on = lane < (int)k;
        uint32_t u = 0, a0 = 0, a1 = 0;
        uint64_t ku = 0;
        bool stuck = false;
        if (on) {
          volatile uint16_t* slot = &qring[(h + lane) & (qcap - 1)];
          uint16_t x;
          uint32_t sp = 0;
          while ((x = *slot) == QB_EMPTY && ++sp < a.spin_max) __builtin_amdgcn_s_sleep(0);
          stuck = x == QB_EMPTY;
          *slot = QB_EMPTY;
          const uint32_t xs = stuck ? 0u : x;
          u = hid[xs];
          // clear the dirty flag; the returned key is the one to relax with
          ku = __hip_atomic_fetch_and(&hkey[xs], ~1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & ~1ull;
          a0 = __builtin_amdgcn_raw_buffer_load_b32(roff, stuck ? 0x80000000u : u * 4u, 0, 0);
          a1 = __builtin_amdgcn_raw_buffer_load_b32(roff, stuck ? 0x80000000u : u * 4u + 4u, 0, 0);
        }
        if (__any(stuck)) {
          if (lane == 0) give_up();
          goto wave_exit;
        }
        if (COUNT) n_pop += __popcll(__ballot(on));
        const uint32_t deg = a1 - a0;
        __builtin_amdgcn_s_waitcnt(0);  // (diagnostics only: the offsets are in)
        const unsigned long long t1 = wclk();
        const uint32_t dmax = __builtin_amdgcn_readlane(wave_incl_max(deg), 63);
        if (COUNT) n_rel += __builtin_amdgcn_readlane(wave_incl_sum(deg), 63);
        for (uint32_t j0 = 0; j0 < dmax; j0 += LA) {
          uint32_t v[LA], sl[LA];
          uint64_t cd[LA];
          bool hs[LA];
#pragma unroll
          for (int c = 0; c < LA; c++) {
            const bool valid = j0 + c < deg;
            const auto r = __builtin_amdgcn_raw_buffer_load_b96(arcs, valid ? (a0 + j0 + c) * 12u : 0x80000000u, 0, 0);
            v[c] = valid ? r[0] : 0u;
            cd[c] = valid ? bkey_relax(ku, r[1], __uint_as_float(r[2])) : ~0ull;
          }
#pragma unroll
          for (int c = 0; c < LA; c++) {
            const uint32_t lat = bkey_lat(cd[c]);
            const bool live = j0 + c < deg && lat != LAT32_SAT && !is_settled(v[c]);
            const uint32_t d = bk_bucket(lat, a.delta, a.dmul) - b;  // >= 0: later than its tail's key
            hs[c] = live && d == 0;
            sl[c] = !live || d == 0 ? 0xFFFFFFFFu : d < R ? ((b + d) & rmask) : far;
          }
          const unsigned long long t2 = wclk();
          append_entries(std::integral_constant<int, LA>(), sl, v, cd, false);
          if (COUNT) {
            wc[2] += t2 - t1;
            wc[3] += wclk() - t2;
          }
#pragma unroll
          for (int c = 0; c < LA; c++) {
            if (!__any(hs[c])) continue;
            uint32_t x;
            const bool app = offer_hash(hs[c], v[c], cd[c], x);
            append_q(app, x);
          }
        }
        if (lane == 0) atomicSub(&hb, 1ull);  // release the claim after this wave's appends
        if (COUNT) {
          wc[1] += t1 - t0;
          wc[4] += wclk() - t0;
        }
      }
      // quiescent: the staged entries and the band's slots are final
      const uint32_t nstg = min(ld(&ctl[STG]), a.stg_cap), nu = ld(&ctl[UCNT]);
      __syncthreads();
      stamp(0);
      if (ld(&ctl[ABORT])) goto wave_exit;
      // ---- C: store the staged entries to the arena; settle the band; free bucket b's chunks; find
      // the next bucket
      for (uint32_t i = tid; i < nstg; i += NT) {
        const uint4 r = stg[i];
        typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
        __builtin_amdgcn_raw_buffer_store_b96((u32x3){r.x, r.y, r.z}, ra, r.w * 12u, 0, 0);
      }
      for (uint32_t i = tid; i < nu; i += NT) {
        const uint32_t x = ulist[i];
        const uint32_t id = hid[x];
        const uint64_t kk = hkey[x];
        atomicOr(&settled[id >> 5], 1u << (id & 31));
        __builtin_amdgcn_raw_buffer_store_b64(
            (uint32_t __attribute__((ext_vector_type(2)))){bkey_loss_bits(kk), bkey_lat(kk)}, rs, id * 8u, 0, 0);
        hid[x] = HID_EMPTY;
        hkey[x] = BKEY_INF;
      }
      if (wv == 0) {
        const uint32_t sb = b & rmask;
        const uint32_t nc = (cnt[sb] + BK_CH - 1) >> BK_CH_LOG;  // <= BK_MAXCH (<= 64 lanes)
        int top = (int)ctl[FTOP];
        top = top < 0 ? 0 : top;
        if (lane < (int)nc) {
          fstack[top + lane] = tab[sb * BK_MAXCH + lane];
          tab[sb * BK_MAXCH + lane] = CH_EMPTY;
        }
        // the next bucket nb: the first non-empty ring slot after b.  The ring holds every entry of
        // the buckets [b, b + R); once a far entry's bucket fm enters [nb, nb + R) -- or the ring is
        // empty -- a far step first moves the far list's entries into the ring relative to
        // min(nb, fm), so that the ring holds every entry of its window again
        const uint64_t m0 = __ballot(lane >= 1 && (uint32_t)lane < R && cnt[(b + lane) & rmask] != 0u);
        const uint64_t m1 = __ballot((uint32_t)lane + 64 < R && cnt[(b + lane + 64) & rmask] != 0u);
        if (lane == 0) {
          ctl[FTOP] = (uint32_t)(top + (int)nc);
          cnt[sb] = 0;
          const uint32_t nb = m0 ? b + (uint32_t)__builtin_ctzll(m0)
                                 : m1 ? b + 64 + (uint32_t)__builtin_ctzll(m1) : NEXT_DONE;
          const uint32_t fm = cnt[far] ? ctl[FARMIN + (far - BK_R)] : NEXT_DONE;
          const bool go_far = fm != NEXT_DONE && (nb == NEXT_DONE || fm < nb || fm - nb < R);
          ctl[NEXT] = go_far ? NEXT_FAR : nb;
          ctl[FMIN] = min(nb, fm);
          ctl[STG] = 0;
          ctl[UCNT] = 0;
          // the queue is empty (head == tail); every wave busy with the next band's load
          hb = ((unsigned long long)ctl[TAIL] << 32) | NW;
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's entry and scratch stores are in L2
      __syncthreads();
      stamp(1);
      const uint32_t nx = ctl[NEXT];
      if (nx == NEXT_DONE) break;
      if (nx == NEXT_FAR) {
        // ---- far step: the far list's entries redistributed over the ring (relative to b0) and the
        // other far list (a settled node's entries are dropped)
        if (COUNT) n_far++;
        const uint32_t fc = cnt[far];
        const uint32_t b0 = ctl[FMIN];
        const uint32_t nfar = far == BK_R ? BK_R + 1 : BK_R;
        for (uint32_t i0 = wv * 64; i0 < fc; i0 += NT) {  // whole waves (append_entries is wave-wide)
          const uint32_t i = i0 + lane;
          uint32_t s = 0xFFFFFFFFu, v = 0;
          uint64_t cd = ~0ull;
          if (i < fc) {
            const uint32_t id = tab[far * BK_MAXCH + (i >> BK_CH_LOG)];
            const uint32_t e = (id << BK_CH_LOG) | (i & (BK_CH - 1));
            const auto r = __builtin_amdgcn_raw_buffer_load_b96(ra, e * 12u, 0, BK_SC1);
            v = r[0];
            cd = ((uint64_t)r[1] << 32) | ((uint64_t)r[2] << 1) | 1ull;
            const uint32_t d = bk_bucket(r[1], a.delta, a.dmul) - b0;
            if (!is_settled(v)) s = d < R ? ((b0 + d) & rmask) : nfar;
          }
          append_entries(std::integral_constant<int, 1>(), &s, &v, &cd, true);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (ld(&ctl[ABORT])) goto wave_exit;
        if (wv == 0) {  // the old far list's chunks back to the free stack
          const uint32_t nc = (fc + BK_CH - 1) >> BK_CH_LOG;
          int top = (int)ctl[FTOP];
          top = top < 0 ? 0 : top;
          if (lane < (int)nc) {
            fstack[top + lane] = tab[far * BK_MAXCH + lane];
            tab[far * BK_MAXCH + lane] = CH_EMPTY;
          }
          if (lane == 0) {
            ctl[FTOP] = (uint32_t)(top + (int)nc);
            cnt[far] = 0;
            ctl[FARMIN + (far - BK_R)] = 0xFFFFFFFFu;
          }
        }
        far = nfar;
        b = b0;
        __syncthreads();
        stamp(2);
      } else {
        b = nx;
      }
    }
    if (COUNT && lane == 0) {
      if (n_rel) atomicAdd(&a.work[bi & 63], n_rel);
      if (a.diag && wv == 0) {
        atomicAdd(&a.diag[0], n_bk);
        atomicAdd(&a.diag[2], n_far);
      }
      if (a.diag) {
        atomicAdd(&a.diag[1], n_app);
        atomicAdd(&a.diag[3], n_pop);
        atomicAdd(&a.diag[8], n_claim);
        for (int k = 0; k < 6; k++) atomicAdd(&a.diag[9 + k], wc[k]);
        if (tid == 0)
          for (int k = 0; k < 3; k++) atomicAdd(&a.diag[4 + k], cyc[k]);
      }
    }
    n_rel = n_app = n_bk = n_far = n_pop = n_claim = 0;
    for (int k = 0; k < 6; k++) wc[k] = 0;
    for (int k = 0; k < 4; k++) cyc[k] = 0;
    stamp(-1);

    // ---- write the row: columns in used order, diagonal = the raw self-loop (graph/mod.rs:210-217);
    // a node never settled (unreachable, or past 2^32 ns) flags the row for the wide kernel
    if (tid == 0) s_item = atomicAdd(a.item_ctr, 1u);  // the next row (read after the row loop's barrier)
    {
      const size_t orow = (size_t)(row - a.row_begin) * a.n_used;
      bool sat = false;
      const uint32_t de = a.self_edge[src];
      const uint64_t d_lat = a.e_lat[de];
      const float d_loss = a.e_loss[de];
      auto cell = [&](uint32_t j, uint32_t vj, uint64_t kk, uint64_t& l, float& f) {
        const bool dg = j == row;
        const bool st = is_settled(vj);
        sat |= !dg && !st;
        l = dg ? d_lat : st ? (kk >> 32) : (uint64_t)LAT32_SAT;
        f = dg ? d_loss : st ? __uint_as_float((uint32_t)kk) : 1.0f;
      };
      if (a.vec_out) {
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        typedef float f32x4 __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc((void*)a.used, 0, (int)(a.n_used * 4u),
                                                                            0x00020000);
        for (uint32_t j = tid * 4; j < a.n_used; j += NT * 4) {
          const auto uv = __builtin_amdgcn_raw_buffer_load_b128(ru, j * 4u, 0, 0);
          uint64_t k4[4];
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, uv[q] * 8u, 0, BK_SC1);
            k4[q] = ((uint64_t)x[1] << 32) | x[0];
          }
          uint64_t l[4];
          float f[4];
#pragma unroll
          for (int q = 0; q < 4; q++) cell(j + q, uv[q], k4[q], l[q], f[q]);
          __builtin_nontemporal_store((u64x2){l[0], l[1]}, (u64x2*)&a.out_lat[orow + j]);
          __builtin_nontemporal_store((u64x2){l[2], l[3]}, (u64x2*)&a.out_lat[orow + j + 2]);
          __builtin_nontemporal_store((f32x4){f[0], f[1], f[2], f[3]}, (f32x4*)&a.out_loss[orow + j]);
        }
      } else {
        for (uint32_t j = tid; j < a.n_used; j += NT) {
          const uint32_t vj = a.used[j];
          const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, vj * 8u, 0, BK_SC1);
          uint64_t l;
          float f;
          cell(j, vj, ((uint64_t)x[1] << 32) | x[0], l, f);
          a.out_lat[orow + j] = l;
          a.out_loss[orow + j] = f;
        }
      }
      if (__any(sat) && lane == 0) a.sat_row[row - a.row_begin] = 1u;
    }
    if (COUNT && a.diag && tid == 0) {
      stamp(3);
      atomicAdd(&a.diag[7], cyc[3]);
      cyc[3] = 0;
    }
  }
wave_exit:;
}

// ---------------------------------------------------------------------------------------------
// Exact bands (Delta <= the smallest arc latency): a candidate is always later than the band it
// comes from, so a band never relaxes into itself.  Its entries are deduplicated once (the
// smallest key per node, in an LDS hash), every node of the band is settled at once, and the
// band's arcs are relaxed arc-parallel: each wave takes 64 of the band's nodes, lays their arcs
// out in consecutive slots (owner lane by scatter + max-scan, sg_sssp.hip's expansion path) and
// reads BD_K x 64 of them per step, consecutive lanes on consecutive arcs of a node.  No queue,
// no dirty flags; a band is three barriers: load, relax, next.  The LDS per row is the settled
// bitmap, the hash and the ring's chunk tables (~39 KB at C5), so four rows share a CU and hide
// each other's round trips.
constexpr uint32_t BD_CH_LOG = 10;
constexpr uint32_t BD_CH = 1u << BD_CH_LOG;  // entries per chunk
constexpr uint32_t BD_MAXCH = 8;            // chunks per bucket: 8,192 entries
constexpr int BD_K = 8;                     // arc slots of 64 a wave reads per step
constexpr int BD_G = 4;                     // entries a lane loads per step
constexpr int BD_NCLS = 17;                 // degree classes: out-degree 0 .. 15, and 16 or more
// A band's appends to a ring slot are staged in LDS, up to BD_E per slot, at their arena order, and
// stored after the band as runs of consecutive entries (a few memory requests per slot instead
// of one per entry); the rest, and far-list entries, are stored at once
constexpr uint32_t BD_E_MAX = 16;
// dynamic LDS: hid[HS] u32, hkey[HS] u64, ulist[HS] u16, settled[nbw] u32, tab[BK_SLOTS][BD_MAXCH] u16,
// cnt[BK_SLOTS] u32, cst[BK_R] u32 (counts at the band's start), fstack[nch] u16, own[NW][64 BD_K] u8,
// stg[BK_R][E] 12 B
struct BdLds {
  size_t o_hkey, o_ul, o_set, o_tab, o_cnt, o_cst, o_fst, o_own, o_stg, bytes;
  __host__ __device__ BdLds(uint32_t n, uint32_t hs, uint32_t nch, uint32_t nw, uint32_t e) {
    o_hkey = (size_t)hs * 4;
    o_ul = o_hkey + (size_t)hs * 8;
    o_set = (o_ul + (size_t)hs * 2 + 7) / 8 * 8;
    o_tab = o_set + ((size_t)(n + 31) / 32 * 4 + 7) / 8 * 8;
    o_cnt = o_tab + (size_t)BK_SLOTS * BD_MAXCH * 2;
    o_cst = o_cnt + (size_t)BK_SLOTS * 4;
    o_fst = o_cst + (e ? (size_t)BK_R * 4 : 0);  // (none without staging: 512 B decide 3 or 4 rows per CU at C5)
    o_own = (o_fst + (size_t)nch * 2 + 15) / 16 * 16;
    o_stg = o_own + (size_t)nw * 64 * BD_K;
    bytes = o_stg + (size_t)BK_R * e * 12;
  }
};

// Cache policies of the band kernel's streams (buffer aux bits: 16 sc1, 2 nt; A/B builds set them).
// Measured at 12,800 C5 rows (r7b-r7d): entry stores sc1 86.8 ms and nt 147.8 against plain 62.3 --
// the L2 merges a bucket list's 12-B appends into whole lines, and must keep them; entry loads nt
// 61.1; scratch stores sc1 63.2.  Without the scratch stores at all (a wrong table) 52.4: the
// settled keys' 8-B stores spread over a row's whole search leave L2 one partial line each.  A
// settled list in their place (whole-line appends, the row's cells scattered at its end) took
// 65.7-70.9 against 56.0-62.3: the end-of-row scatter costs more than it saves; the same list
// put in column order by a counting sort over column blocks and written block by block from LDS
// (no scattered store at all) 64.1-64.3 against 61.5-61.6: three passes over the list cost more.
#ifndef BD_ST_POL
#define BD_ST_POL 0  // arena entry stores
#endif
#ifndef BD_LD_POL
#define BD_LD_POL (BK_SC1 | 2)  // arena entry loads: read once
#endif
#ifndef BD_SCR_POL
#define BD_SCR_POL 0  // settled keys to the scratch row
#endif
#ifndef BD_ARC_POL
#define BD_ARC_POL 0  // arc records
#endif
template <bool COUNT, int NT>
__global__ void __launch_bounds__(NT) k_sssp_band(BkArgs a) {
  constexpr uint32_t NW = NT / 64;
  extern __shared__ __align__(16) unsigned char smem[];
  const uint32_t HS = 1u << a.hs_log2, hmask = HS - 1;
  const uint32_t n = a.n, R = a.ring, rmask = R - 1;
  const uint32_t E = a.stg_cap;  // staged entries per ring slot and band (0: none)
  const BdLds L(n, HS, a.nch, NW, E);
  uint32_t* hid = (uint32_t*)smem;
  unsigned long long* hkey = (unsigned long long*)(smem + L.o_hkey);
  uint16_t* ulist = (uint16_t*)(smem + L.o_ul);
  uint32_t* settled = (uint32_t*)(smem + L.o_set);
  uint16_t* tab = (uint16_t*)(smem + L.o_tab);
  uint32_t* cnt = (uint32_t*)(smem + L.o_cnt);
  uint16_t* fstack = (uint16_t*)(smem + L.o_fst);
  uint32_t* cst = (uint32_t*)(smem + L.o_cst);
  uint32_t* stg = (uint32_t*)(smem + L.o_stg);
  const uint32_t nbw = (n + 31) / 32;
  constexpr int ABORT = 2, FTOP = 3, FBUMP = 4, FARMIN = 7, UCNT = 10, OVF = 11;
  const uint32_t ulim = HS - HS / 4;  // nodes a (sub-)band may hold: past it the band splits
  __shared__ uint32_t ctl[16];
  __shared__ uint32_t s_item;
  __shared__ uint32_t s_cls[2 * BD_NCLS];  // degree classes: first internal id, first arc
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint8_t* ow = (uint8_t*)(smem + L.o_own) + wv * 64 * BD_K;
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  constexpr uint64_t KINF = KEY_INF;  // packed (latency << 32) | bits(loss), no flag

  for (uint32_t i = tid; i < HS; i += NT) {
    hid[i] = HID_EMPTY;
    hkey[i] = KINF;
  }
  for (uint32_t i = tid; i < BK_SLOTS * BD_MAXCH; i += NT) tab[i] = CH_EMPTY;
  for (uint32_t i = tid; i < BK_SLOTS; i += NT) cnt[i] = 0;
  if (tid < 16) ctl[tid] = tid == FARMIN || tid == FARMIN + 1 ? NONE : 0u;
  for (uint32_t i = lane; i < 64 * BD_K; i += 64) ow[i] = 0;
  if (tid < 2 * BD_NCLS) s_cls[tid] = a.cls[tid];
  const size_t ent0 = (size_t)blockIdx.x * a.arena_words;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)(a.arena + ent0), 0,
                                                                      (int)(a.nch * BD_CH * 12u), 0x00020000);
  unsigned long long* scr = a.scratch + (size_t)blockIdx.x * a.scr_stride;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)scr, 0, (int)(n * 8u), 0x00020000);
  const __amdgpu_buffer_rsrc_t arcs = __builtin_amdgcn_make_buffer_rsrc((void*)a.out_arc, 0, (int)(a.n_arcs * 12u),
                                                                        0x00020000);
  const __amdgpu_buffer_rsrc_t roff = __builtin_amdgcn_make_buffer_rsrc((void*)a.hi_off, 0, (int)((n + 1) * 4u),
                                                                        0x00020000);
  const bool use_filt = a.filt != nullptr;
  const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(use_filt ? a.filt + (size_t)blockIdx.x * a.filt_stride : a.filt), 0, (int)a.filt_stride, 0x00020000);
  if (tid == 0) s_item = atomicAdd(a.item_ctr, 1u);
  auto ld = [](uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
  auto is_settled = [&](uint32_t v) { return (settled[v >> 5] >> (v & 31)) & 1u; };
  uint32_t row = 0;
  auto give_up = [&]() {
    if (atomicExch(&ctl[ABORT], 1u) == 0u) {
      a.sat_row[row - a.row_begin] = 2u;
      __threadfence();
      if (atomicAdd(&a.item_ctr[1], 1u) == gridDim.x - 1) {
        const uint32_t c = __hip_atomic_load(&a.item_ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t i = min(c, a.rows); i < a.rows; i++) a.sat_row[i] = 2u;
      }
    }
  };
  unsigned long long n_rel = 0, n_app = 0, n_bk = 0, n_far = 0, n_pop = 0;
  unsigned long long cyc[4] = {0, 0, 0, 0};  // COUNT, thread 0: cycles in load, relax, next, output
  unsigned long long t_mark = 0;
  unsigned long long wc[4] = {0, 0, 0, 0};  // COUNT, thread 0: relax sub-steps (offsets, arcs, appends, store wait)
  unsigned long long wl[3] = {0, 0, 0};     // COUNT, thread 0: load sub-steps (entry loads, hash, barrier wait)
  auto wclk = [&]() -> unsigned long long { return COUNT ? clock64() : 0ull; };
  auto stamp = [&](int k) {
    if (COUNT && tid == 0) {
      const unsigned long long t = clock64();
      if (k >= 0) cyc[k] += t - t_mark;
      t_mark = t;
    }
  };
  // node v's hash slot, inserted (and listed) if absent; HS: the table is full.  Past ulim nodes
  // the pass is flagged (OVF) and redone over the band's lower half (see the band loop); once it
  // is flagged nothing more is inserted (HS + 1: skip), so the table never fills
  auto hash_slot = [&](uint32_t v) -> uint32_t {
    uint32_t h = (v * 0x9E3779B1u) >> (32 - a.hs_log2);
    for (uint32_t p = 0; p < HS; p++) {
      const uint32_t id = ld(&hid[h]);
      if (id == v) return h;
      if (id == HID_EMPTY) {
        if (ld(&ctl[OVF])) return HS + 1;
        const uint32_t o = atomicCAS(&hid[h], HID_EMPTY, v);
        if (o == HID_EMPTY) {
          const uint32_t k = atomicAdd(&ctl[UCNT], 1u);
          if (k < ulim) ulist[k] = (uint16_t)h;
          else ctl[OVF] = 1u;
          return h;
        }
        if (o == v) return h;
      }
      h = (h + 1) & hmask;
    }
    return HS;
  };
  auto alloc_chunk = [&]() -> uint32_t {
    const int t = atomicSub((int*)&ctl[FTOP], 1) - 1;
    if (t >= 0) return fstack[t];
    const uint32_t id = atomicAdd(&ctl[FBUMP], 1u);
    if (id >= a.nch) {
      give_up();
      return 0u;
    }
    return id;
  };
  // append entries (node, packed key) to slots s[c] (>= BK_SLOTS: none); `stage`: a ring slot's first
  // E appends of the band go to the LDS staging (stored after the band), the rest straight to the arena
  auto append = [&](auto nk, const uint32_t* s, const uint32_t* v, const uint64_t* key, bool stage) {
    constexpr int NK = decltype(nk)::value;
    uint32_t pos[NK];
#pragma unroll
    for (int c = 0; c < NK; c++) pos[c] = s[c] < BK_SLOTS ? atomicAdd(&cnt[s[c]], 1u) : 0u;
#pragma unroll
    for (int c = 0; c < NK; c++)
      if (s[c] >= BK_R && s[c] < BK_SLOTS)
        atomicMin(&ctl[FARMIN + (s[c] - BK_R)], bk_bucket((uint32_t)(key[c] >> 32), a.delta, a.dmul));
#pragma unroll
    for (int c = 0; c < NK; c++) {
      if (s[c] < BK_SLOTS && (pos[c] >> BD_CH_LOG) < BD_MAXCH && (pos[c] & (BD_CH - 1)) == 0) {
        const uint32_t id = alloc_chunk();
        __hip_atomic_store(&tab[s[c] * BD_MAXCH + (pos[c] >> BD_CH_LOG)], (uint16_t)id, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
#pragma unroll
    for (int c = 0; c < NK; c++) {
      if (s[c] >= BK_SLOTS) continue;
      if ((pos[c] >> BD_CH_LOG) >= BD_MAXCH) {
        give_up();
        continue;
      }
      uint16_t* tp = &tab[s[c] * BD_MAXCH + (pos[c] >> BD_CH_LOG)];
      uint16_t id;
      uint32_t sp = 0;
      while ((id = __hip_atomic_load(tp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) == CH_EMPTY &&
             ++sp < a.spin_max)
        __builtin_amdgcn_s_sleep(0);
      if (id == CH_EMPTY) {
        give_up();
        continue;
      }
      const uint32_t k = E && stage && s[c] < BK_R ? pos[c] - cst[s[c]] : E;
      if (k < E) {  // staged at its arena order, stored after the band
        uint32_t* q = stg + (s[c] * E + k) * 3;
        q[0] = v[c];
        q[1] = (uint32_t)(key[c] >> 32);
        q[2] = (uint32_t)key[c];
        continue;
      }
      typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
      const uint32_t e = ((uint32_t)id << BD_CH_LOG) | (pos[c] & (BD_CH - 1));
      __builtin_amdgcn_raw_buffer_store_b96((u32x3){v[c], (uint32_t)(key[c] >> 32), (uint32_t)key[c]}, ra, e * 12u, 0,
                                            BD_ST_POL);
    }
    if (COUNT) {
#pragma unroll
      for (int c = 0; c < NK; c++) n_app += __popcll(__ballot(s[c] < BK_SLOTS));
    }
  };
  // the slot an entry of bucket bk goes to while bucket b is processed (b <= bk)
  auto slot_of = [&](uint32_t bk, uint32_t b, uint32_t far) -> uint32_t {
    const uint32_t d = bk - b;
    return d < R ? ((b + d) & rmask) : far;
  };
  // free a slot's chunks (one wave)
  auto free_slot = [&](uint32_t sb) {
    const uint32_t nc = (cnt[sb] + BD_CH - 1) >> BD_CH_LOG;  // <= BD_MAXCH
    int top = (int)ctl[FTOP];
    top = top < 0 ? 0 : top;
    if (lane < (int)nc) {
      fstack[top + lane] = tab[sb * BD_MAXCH + lane];
      tab[sb * BD_MAXCH + lane] = CH_EMPTY;
    }
    if (lane == 0) {
      ctl[FTOP] = (uint32_t)(top + (int)nc);
      cnt[sb] = 0;
    }
  };

  for (;;) {  // rows
    __syncthreads();
    const uint32_t bi = s_item;
    if (bi >= a.rows) break;
    row = a.row_begin + bi;
    const uint32_t src = a.used_key[row];  // (the degree-class id)
    for (uint32_t i = tid; i < nbw; i += NT) settled[i] = 0u;
    if (use_filt) {  // the filter starts empty; in L2 before any read of this row (the barrier below)
      for (uint32_t i = tid * 16u; i < a.filt_stride; i += NT * 16u)
        __builtin_amdgcn_raw_buffer_store_b128((uint32_t __attribute__((ext_vector_type(4)))){0u, 0u, 0u, 0u}, rf, i,
                                               0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (tid == 0) {  // PathProperties::default() at the source: band 0
      const uint32_t h = (src * 0x9E3779B1u) >> (32 - a.hs_log2);
      hid[h] = src;
      hkey[h] = 0ull;
      ulist[0] = (uint16_t)h;
      ctl[UCNT] = 1;
    }
    uint32_t b = 0, far = BK_R;
    // the (sub-)band's latencies [sub_lo, sub_hi): the whole band [b delta, (b + 1) delta), or its
    // lower part when the band holds more nodes than the hash takes (then the rest follows, from the
    // same bucket list: a candidate is at least w_min >= delta past its tail, so no relaxation of
    // the band lands in it)
    uint64_t sub_lo = 0, sub_hi = a.delta;
    __syncthreads();
    stamp(-1);
    for (;;) {  // bands
      if (COUNT) n_bk++;
      // ---- load: bucket b's entries into the hash, the smallest key per node (a settled node's are stale)
      if (E)  // the ring's counts before this band's appends (the staging's arena positions)
        for (uint32_t q = tid; q < R; q += NT) cst[q] = cnt[q];
      {
        const uint32_t sb = b & rmask, c = cnt[sb];
        unsigned long long l0 = wclk();
        for (uint32_t i0 = tid; i0 < c; i0 += NT * BD_G) {
          uint32_t v[BD_G];
          uint64_t key[BD_G];
#pragma unroll
          for (int g = 0; g < BD_G; g++) {
            const uint32_t i = i0 + g * NT;
            const bool on = i < c;
            const uint32_t id = on ? tab[sb * BD_MAXCH + (i >> BD_CH_LOG)] : 0u;
            const uint32_t e = (id << BD_CH_LOG) | (i & (BD_CH - 1));
            const auto r = __builtin_amdgcn_raw_buffer_load_b96(ra, on ? e * 12u : 0x80000000u, 0, BD_LD_POL);
            v[g] = on && (uint64_t)r[1] < sub_hi ? r[0] : NONE;  // (past the sub-band: a later pass)
            key[g] = ((uint64_t)r[1] << 32) | r[2];
          }
          if (COUNT) {
            __builtin_amdgcn_s_waitcnt(0);
            const unsigned long long l1 = wclk();
            wl[0] += l1 - l0;
            l0 = l1;
          }
          // (Two buckets per load step -- both lists into the hash, bucket b relaxed with its candidates
          // for bucket b + 1 inserted, then bucket b + 1 -- measured slower, 74.1 against 59.7 ms, r8q: the
          // load step's hash time grew 6.1k -> 25.9k cycles for twice the entries.)
          // (the thread's BD_G entries hashed together -- settled filter, first probes, CASes in flight at
          // once, one UCNT add per wave -- with the appends' chunk-id reads batched the same way measured
          // slower: 60.7 against 59.6 ms, r8l; the load step's hash time rose 6.2k -> 7.2k cycles: the
          // LDS pipe, shared by four rows, not the round trips, sets it)
          uint32_t x[BD_G];
#pragma unroll
          for (int g = 0; g < BD_G; g++) {
            x[g] = v[g] != NONE && !is_settled(v[g]) ? hash_slot(v[g]) : NONE;
            if (x[g] == HS) give_up();
          }
#pragma unroll
          for (int g = 0; g < BD_G; g++)
            if (x[g] < HS)
              (void)__hip_atomic_fetch_min(&hkey[x[g]], (unsigned long long)key[g], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
          if (COUNT) {
            __builtin_amdgcn_s_waitcnt(0);
            const unsigned long long l1 = wclk();
            wl[1] += l1 - l0;
            l0 = l1;
          }
        }
        if (COUNT) l0 = wclk();
        __syncthreads();
        if (COUNT) wl[2] += wclk() - l0;
      }
      stamp(0);
      if (ld(&ctl[ABORT])) goto wave_exit;
      if (ld(&ctl[OVF])) {  // (uniform) too many nodes: the lower half of the (sub-)band again
        for (uint32_t i = tid; i < HS; i += NT) {
          hid[i] = HID_EMPTY;
          hkey[i] = KINF;
        }
        __syncthreads();  // every wave has read OVF
        if (tid == 0) {
          ctl[OVF] = 0u;
          ctl[UCNT] = 0u;
        }
        sub_hi = sub_lo + (sub_hi - sub_lo) / 2;
        if (sub_hi <= sub_lo || E) give_up();  // (a 1-ns band, or staging on: the wide kernel)
        if (COUNT && a.diag && tid == 0) atomicAdd(&a.diag[15], 1ull);  // band splits
        __syncthreads();
        if (ld(&ctl[ABORT])) goto wave_exit;
        continue;
      }
      // ---- relax: the band's nodes are final; settle them and relax their arcs arc-parallel
      {
        const uint32_t U = ctl[UCNT];
        const uint32_t bm = b % 255u;  // (the append filter's buckets are kept mod 255)
        if (COUNT && tid == 0) n_pop += U;
        const uint32_t npw = a.npw;  // band nodes per wave and step
        for (uint32_t i0 = wv * npw; i0 < U; i0 += NW * npw) {  // whole waves
          const uint32_t i = i0 + lane;
          const bool on = (uint32_t)lane < npw && i < U;
          const uint32_t x = on ? ulist[i] : 0u;
          const uint32_t u = on ? hid[x] : 0u;
          const uint64_t ku = on ? hkey[x] : 0ull;
          // the node's arc range from its degree class, no memory round trip: class k < 16 holds the
          // nodes of out-degree k, arcs first[k] .. in id order; class 16 (degree >= 16) reads its offsets
          uint32_t k = 0;
#pragma unroll
          for (int c = 1; c < BD_NCLS; c++) k += u >= s_cls[c] ? 1u : 0u;
          uint32_t a0 = s_cls[BD_NCLS + k] + (u - s_cls[k]) * k, a1 = a0 + k;
          if (__builtin_amdgcn_ballot_w64(on && k == BD_NCLS - 1)) {
            const bool hi = on && k == BD_NCLS - 1;
            const auto ar = __builtin_amdgcn_raw_buffer_load_b64(roff, hi ? (u - s_cls[BD_NCLS - 1]) * 4u : 0x80000000u, 0, 0);
            if (hi) {
              a0 = ar[0];
              a1 = ar[1];
            }
          }
          if (!on) a0 = a1 = 0u;
          if (on) {
            atomicOr(&settled[u >> 5], 1u << (u & 31));
            hid[x] = HID_EMPTY;
            hkey[x] = KINF;
          }
          const unsigned long long q0 = wclk();
          const uint32_t deg = a1 - a0;
          if (COUNT) __builtin_amdgcn_s_waitcnt(0);  // (diagnostics: the offsets are in)
          const unsigned long long q1 = wclk();
          if (COUNT) wc[0] += q1 - q0;
          // arcs [ea0, ea0 + edeg) of each lane's node, arc-parallel: the wave's arcs in consecutive
          // slots, KX chunks of 64 at once, consecutive lanes on consecutive arcs of a node
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
              uint32_t o[KX];
#pragma unroll
              for (int c = 0; c < KX; c++) {
                const uint32_t hd = ow[c * 64 + lane];
                ow[c * 64 + lane] = 0;
                const uint32_t mx = max(wave_incl_max(hd), carry);
                carry = __builtin_amdgcn_readlane(mx, 63);
                o[c] = mx - 1;
              }
              uint32_t v[KX], s[KX];
              uint64_t cd[KX];
#pragma unroll
              for (int c = 0; c < KX; c++) {
                const uint32_t sl = t0 + c * 64 + lane;
                const bool valid = sl < T;
                const uint32_t ai = __shfl(ea0, (int)o[c]) + sl - __shfl(base, (int)o[c]);
                const auto r = __builtin_amdgcn_raw_buffer_load_b96(arcs, valid ? ai * 12u : 0x80000000u, 0, BD_ARC_POL);
                const uint32_t klo = __shfl((uint32_t)ku, (int)o[c]), khi = __shfl((uint32_t)(ku >> 32), (int)o[c]);
                v[c] = r[0];
                cd[c] = valid ? relax32(((uint64_t)khi << 32) | klo, r[1], __uint_as_float(r[2])) : KINF;
              }
#pragma unroll
              for (int c = 0; c < KX; c++) {
                const uint32_t lat = key_lat(cd[c]);
                const bool live = lat != LAT32_SAT && !is_settled(v[c]);
                s[c] = live ? slot_of(bk_bucket(lat, a.delta, a.dmul), b, far) : NONE;
              }
              if (use_filt) {
                // The append filter: a candidate in a later bucket than one already appended for its
                // node cannot be that node's key (its latency is larger), so it is dropped.  Each node
                // keeps 1 + (its best appended bucket mod 255); while a node is unsettled that bucket
                // is >= b, and it is recorded only within b + 254, so it decodes relative to b.  Reads
                // are L2-served (sc1) and racy: a stale value is an older, larger bucket of a real
                // entry, or none, so it only lets more candidates through.  The values of the row
                // before were cleared before this row's first barrier.
                uint32_t fv[KX], d[KX];
#pragma unroll
                for (int c = 0; c < KX; c++) {
                  d[c] = s[c] != NONE ? bk_bucket(key_lat(cd[c]), a.delta, a.dmul) - b : 0u;
                  fv[c] = __builtin_amdgcn_raw_buffer_load_b8(rf, s[c] != NONE ? v[c] : 0x80000000u, 0, BK_SC1);
                }
#pragma unroll
                for (int c = 0; c < KX; c++) {
                  if (s[c] == NONE) continue;
                  const uint32_t e = fv[c];
                  const uint32_t rel = e == 0u ? 0xFFFFFFFFu : (e - 1u >= bm ? e - 1u - bm : e - 1u + 255u - bm);
                  if (d[c] > rel) {
                    s[c] = NONE;  // later than an appended candidate of its node
                  } else if (d[c] < rel && d[c] < 255u) {
                    const uint32_t t = bm + d[c];
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(1u + (t >= 255u ? t - 255u : t)), rf, v[c], 0, 0);
                  }
                }
              }
              const unsigned long long q2 = wclk();
              append(std::integral_constant<int, KX>(), s, v, cd, true);
              if (COUNT) wc[2] += wclk() - q2;
            }
          };
          // (a lane walking its own node's first 8 arcs, with the rest arc-parallel as k_sssp_lds does,
          // measured slower here: 71.1 against 61.7 ms at 12,800 C5 rows, r8a -- 64 lines per load.
          // Reading bucket b + 1's first entries behind the arc loads, for the next load step: 56.2
          // against 54.5 ms, r8i -- that step is its hash inserts and the barrier, not the loads)
          expand(std::integral_constant<int, BD_K>(), a0, deg);
          if (COUNT) wc[1] += wclk() - q1;
          // the settled key to the scratch row, after the node's arcs (before them, or with a full wait
          // after the offsets as before r8, measured the same: 61.5-61.6 ms, r8c)
          if (on)
            __builtin_amdgcn_raw_buffer_store_b64(
                (uint32_t __attribute__((ext_vector_type(2)))){(uint32_t)ku, (uint32_t)(ku >> 32)}, rs, u * 8u, 0,
                BD_SCR_POL);
        }
      }
      if (E) __syncthreads();  // every append staged
      // the staged runs: slot q's entries cst[q] .. cst[q] + min(its appends, E), consecutive threads on
      // consecutive entries of a slot
      for (uint32_t t = tid; t < R * E; t += NT) {
        const uint32_t q = t / E, k = t - q * E;
        if (k >= cnt[q] - cst[q]) continue;
        const uint32_t pos = cst[q] + k;
        const uint32_t id = tab[q * BD_MAXCH + (pos >> BD_CH_LOG)];
        const uint32_t* r = stg + t * 3;
        typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
        const uint32_t e = (id << BD_CH_LOG) | (pos & (BD_CH - 1));
        __builtin_amdgcn_raw_buffer_store_b96((u32x3){r[0], r[1], r[2]}, ra, e * 12u, 0, 0);
      }
      {
        const unsigned long long q4 = wclk();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the entries and scratch keys are in L2
        if (COUNT) wc[3] += wclk() - q4;
      }
      __syncthreads();
      stamp(1);
      if (ld(&ctl[ABORT])) goto wave_exit;
      if (sub_hi < (uint64_t)b * a.delta + a.delta) {  // the band's next sub-band, from the same list
        if (tid == 0) ctl[UCNT] = 0;
        sub_lo = sub_hi;
        sub_hi = (uint64_t)b * a.delta + a.delta;
        __syncthreads();
        continue;
      }
      // ---- next band: the first non-empty ring slot after b, or a far step (sg_bucket.hip k_sssp_bucket)
      uint32_t nb, fm;
      {
        const uint64_t m0 = __ballot(lane >= 1 && (uint32_t)lane < R && cnt[(b + lane) & rmask] != 0u);
        const uint64_t m1 = __ballot((uint32_t)lane + 64 < R && cnt[(b + lane + 64) & rmask] != 0u);
        nb = m0 ? b + (uint32_t)__builtin_ctzll(m0) : m1 ? b + 64 + (uint32_t)__builtin_ctzll(m1) : NONE;
        fm = cnt[far] ? ctl[FARMIN + (far - BK_R)] : NONE;
      }
      __syncthreads();  // every wave has read the counts and the band size
      if (wv == 0) free_slot(b & rmask);
      if (tid == 0) ctl[UCNT] = 0;
      const bool go_far = fm != NONE && (nb == NONE || fm < nb || fm - nb < R);
      if (!go_far && nb == NONE) break;
      __syncthreads();  // the free stack settled before any append; the band count reset before any load
      if (go_far) {
        // ---- far step: the far list's entries over the ring (relative to b0) and the other far list
        if (COUNT) n_far++;
        const uint32_t b0 = min(nb, fm), fc = cnt[far];
        const uint32_t nfar = far == BK_R ? BK_R + 1 : BK_R;
        for (uint32_t i0 = wv * 64; i0 < fc; i0 += NT) {  // whole waves
          const uint32_t i = i0 + lane;
          uint32_t s = NONE, v = 0;
          uint64_t key = KINF;
          if (i < fc) {
            const uint32_t id = tab[far * BD_MAXCH + (i >> BD_CH_LOG)];
            const uint32_t e = (id << BD_CH_LOG) | (i & (BD_CH - 1));
            const auto r = __builtin_amdgcn_raw_buffer_load_b96(ra, e * 12u, 0, BK_SC1);
            v = r[0];
            key = ((uint64_t)r[1] << 32) | r[2];
            if (!is_settled(v)) s = slot_of(bk_bucket(r[1], a.delta, a.dmul), b0, nfar);
          }
          append(std::integral_constant<int, 1>(), &s, &v, &key, false);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (ld(&ctl[ABORT])) goto wave_exit;
        if (wv == 0) {
          free_slot(far);
          if (lane == 0) ctl[FARMIN + (far - BK_R)] = NONE;
        }
        far = nfar;
        b = b0;
        __syncthreads();  // the old far list freed before any append
      } else {
        b = nb;
      }
      sub_lo = (uint64_t)b * a.delta;
      sub_hi = sub_lo + a.delta;
      stamp(2);
    }
    if (COUNT && lane == 0) {
      if (n_rel) atomicAdd(&a.work[bi & 63], n_rel);
      if (a.diag) {
        atomicAdd(&a.diag[1], n_app);
        if (tid == 0) {
          atomicAdd(&a.diag[0], n_bk);
          atomicAdd(&a.diag[2], n_far);
          atomicAdd(&a.diag[3], n_pop);
          for (int k = 0; k < 3; k++) atomicAdd(&a.diag[4 + k], cyc[k]);
          for (int k = 0; k < 4; k++) atomicAdd(&a.diag[9 + k], wc[k]);
          atomicAdd(&a.diag[8], wl[0]);
          atomicAdd(&a.diag[13], wl[1]);
          atomicAdd(&a.diag[14], wl[2]);
        }
      }
    }
    n_rel = n_app = n_bk = n_far = n_pop = 0;
    for (int k = 0; k < 4; k++) cyc[k] = wc[k] = 0;
    wl[0] = wl[1] = wl[2] = 0;
    stamp(-1);
    // ---- write the row (as k_sssp_bucket)
    if (tid == 0) s_item = atomicAdd(a.item_ctr, 1u);
    {
      const size_t orow = (size_t)(row - a.row_begin) * a.n_used;
      bool sat = false;
      const uint32_t de = a.self_edge[a.used[row]];
      const uint64_t d_lat = a.e_lat[de];
      const float d_loss = a.e_loss[de];
      auto cell = [&](uint32_t j, uint32_t vj, uint64_t kk, uint64_t& l, float& f) {
        const bool dg = j == row;
        const bool st = is_settled(vj);
        sat |= !dg && !st;
        l = dg ? d_lat : st ? (kk >> 32) : (uint64_t)LAT32_SAT;
        f = dg ? d_loss : st ? __uint_as_float((uint32_t)kk) : 1.0f;
      };
      if (a.vec_out) {
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        typedef float f32x4 __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc((void*)a.used_key, 0, (int)(a.n_used * 4u),
                                                                            0x00020000);
        for (uint32_t j = tid * 4; j < a.n_used; j += NT * 4) {
          const auto uv = __builtin_amdgcn_raw_buffer_load_b128(ru, j * 4u, 0, 0);
          uint64_t k4[4];
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const auto xx = __builtin_amdgcn_raw_buffer_load_b64(rs, uv[q] * 8u, 0, BK_SC1);
            k4[q] = ((uint64_t)xx[1] << 32) | xx[0];
          }
          uint64_t l[4];
          float f[4];
#pragma unroll
          for (int q = 0; q < 4; q++) cell(j + q, uv[q], k4[q], l[q], f[q]);
          __builtin_nontemporal_store((u64x2){l[0], l[1]}, (u64x2*)&a.out_lat[orow + j]);
          __builtin_nontemporal_store((u64x2){l[2], l[3]}, (u64x2*)&a.out_lat[orow + j + 2]);
          __builtin_nontemporal_store((f32x4){f[0], f[1], f[2], f[3]}, (f32x4*)&a.out_loss[orow + j]);
        }
      } else {
        for (uint32_t j = tid; j < a.n_used; j += NT) {
          const uint32_t vj = a.used_key[j];
          const auto xx = __builtin_amdgcn_raw_buffer_load_b64(rs, vj * 8u, 0, BK_SC1);
          uint64_t l;
          float f;
          cell(j, vj, ((uint64_t)xx[1] << 32) | xx[0], l, f);
          a.out_lat[orow + j] = l;
          a.out_loss[orow + j] = f;
        }
      }
      if (__any(sat) && lane == 0) a.sat_row[row - a.row_begin] = 1u;
    }
    if (COUNT && a.diag && tid == 0) {
      stamp(3);
      atomicAdd(&a.diag[7], cyc[3]);
      cyc[3] = 0;
    }
  }
wave_exit:;
}

// ---------------------------------------------------------------------------------------------
// The degree-class numbering of a graph for k_sssp_band (built once per sg_net, kept in the
// context's workspace): nodes sorted by out-degree class (0 .. 15, and 16 or more), in node order
// within a class, and the out-arcs laid out in that order.  A node's arc range is then arithmetic
// -- class k < 16 starts at arc first_arc[k], node i of it at first_arc[k] + i k -- so the search
// settles a node without reading its offsets; class 16 keeps an offsets array.  Measured at C5
// (12,800 rows): 60.9-61.0 against 61.5 ms (profiles/r05/ab_c5_band_classes_r8f.txt).  (A wrong-
// table diagnostic with no offsets load and every degree 8 ran 9 % faster, ab_c5_band_offsets_r8e.txt:
// most of that came from equal degrees -- one step of arc slots per wave, see BkArgs::npw.)
constexpr uint32_t BC_T = 1024;
__global__ void __launch_bounds__(BC_T) k_band_classes(const uint32_t* __restrict__ out_off, uint32_t n,
                                                       uint32_t* __restrict__ perm, uint32_t* __restrict__ nbase,
                                                       uint32_t* __restrict__ hi_off, uint32_t* __restrict__ cls) {
  __shared__ uint32_t cnt[BD_NCLS][BC_T];  // per thread: nodes of each class in its node range
  __shared__ uint32_t hdeg[BC_T];           // per thread: arcs of its class-16 nodes
  __shared__ uint32_t wsum[BD_NCLS + 1][BC_T / 64];
  __shared__ uint32_t first[BD_NCLS + 1], farc[BD_NCLS + 1];
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t per = (n + BC_T - 1) / BC_T, v0 = min(n, t * per), v1 = min(n, v0 + per);
  for (int k = 0; k < BD_NCLS; k++) cnt[k][t] = 0;
  uint32_t hs = 0;
  for (uint32_t v = v0; v < v1; v++) {
    const uint32_t d = out_off[v + 1] - out_off[v];
    const uint32_t k = min(d, (uint32_t)BD_NCLS - 1);
    cnt[k][t]++;
    if (k == BD_NCLS - 1) hs += d;
  }
  hdeg[t] = hs;
  // exclusive scans over the threads, per class and of the class-16 arcs (row BD_NCLS)
  uint32_t ex[BD_NCLS + 1];
#pragma unroll
  for (int k = 0; k <= BD_NCLS; k++) {
    const uint32_t x = k < BD_NCLS ? cnt[k][t] : hdeg[t];
    const uint32_t inc = wave_incl_sum(x);
    ex[k] = inc - x;
    if (lane == 63) wsum[k][wv] = inc;
  }
  __syncthreads();
  if (t <= BD_NCLS) {  // wave totals -> wave offsets, in place; the class totals
    uint32_t acc = 0;
    for (uint32_t w = 0; w < BC_T / 64; w++) {
      const uint32_t x = wsum[t][w];
      wsum[t][w] = acc;
      acc += x;
    }
    first[t] = acc;  // (for now: the total)
  }
  __syncthreads();
  if (t == 0) {
    uint32_t id = 0, arc = 0;
    for (int k = 0; k < BD_NCLS; k++) {
      const uint32_t c = first[k];
      first[k] = id;
      farc[k] = arc;
      id += c;
      arc += k < BD_NCLS - 1 ? c * (uint32_t)k : first[BD_NCLS];  // class 16: its arcs' total
    }
    first[BD_NCLS] = id;  // = n
    farc[BD_NCLS] = arc;  // = the arcs
  }
  __syncthreads();
  uint32_t pos[BD_NCLS];
#pragma unroll
  for (int k = 0; k < BD_NCLS; k++) pos[k] = first[k] + wsum[k][wv] + ex[k];
  uint32_t hp = farc[BD_NCLS - 1] + wsum[BD_NCLS][wv] + ex[BD_NCLS];
  for (uint32_t v = v0; v < v1; v++) {
    const uint32_t d = out_off[v + 1] - out_off[v];
    const uint32_t k = min(d, (uint32_t)BD_NCLS - 1);
    uint32_t id = 0;
#pragma unroll
    for (int c = 0; c < BD_NCLS; c++)
      if ((uint32_t)c == k) id = pos[c]++;
    perm[v] = id;
    if (k < BD_NCLS - 1) {
      nbase[v] = farc[k] + (id - first[k]) * k;
    } else {
      hi_off[id - first[BD_NCLS - 1]] = hp;
      nbase[v] = hp;
      hp += d;
    }
  }
  if (t == 0) hi_off[first[BD_NCLS] - first[BD_NCLS - 1]] = farc[BD_NCLS];
  if (t < BD_NCLS) {
    cls[t] = first[t];
    cls[BD_NCLS + t] = farc[t];
  }
}

// the out-arcs in the degree-class order, heads renumbered (one thread per node)
__global__ void k_band_arcs(const uint32_t* __restrict__ out_off, const uint32_t* __restrict__ out_arc, uint32_t n,
                            const uint32_t* __restrict__ perm, const uint32_t* __restrict__ nbase,
                            uint32_t* __restrict__ arc) {
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
    const uint32_t a0 = out_off[v], d = out_off[v + 1] - a0, b = nbase[v];
    for (uint32_t j = 0; j < d; j++) {
      const uint32_t* r = out_arc + (size_t)(a0 + j) * 3;
      uint32_t* w = arc + (size_t)(b + j) * 3;
      w[0] = perm[r[0]];
      w[1] = r[1];
      w[2] = r[2];
    }
  }
}

// a used list in the degree-class numbering
__global__ void k_band_used(const uint32_t* __restrict__ used, uint32_t n_used, const uint32_t* __restrict__ perm,
                            uint32_t* __restrict__ out) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n_used; j += gridDim.x * blockDim.x)
    out[j] = perm[used[j]];
}

// The launch shape (env knobs are for tests and A/B runs): threads per workgroup (SG_BUCKET_THREADS:
// 256, the default, or 1024), log2 of the hash slots (SG_BUCKET_HASH; small tables give up), arena
// chunks per workgroup (SG_BUCKET_CHUNKS; small arenas give up).  Rows in flight per CU follow from
// the LDS: a band step is a chain of dependent round trips (entries, arcs, stores) over a few
// hundred nodes, so several rows per CU hide each other's waits.
struct BkShape {
  uint32_t nt, hs_log2, nch;
};
static int bk_env(const char* name, int dflt) {
  const char* s = getenv(name);
  return s && *s ? atoi(s) : dflt;
}
static BkShape bk_shape() {
  BkShape k;
  k.nt = bk_env("SG_BUCKET_THREADS", 256) == 1024 ? 1024u : 256u;
  k.hs_log2 = (uint32_t)std::max(6, std::min(14, bk_env("SG_BUCKET_HASH", k.nt == 1024 ? 12 : 11)));
  k.nch = (uint32_t)std::max(4, std::min(65534, bk_env("SG_BUCKET_CHUNKS", 1024)));
  return k;
}
static size_t bk_fixed_lds(uint32_t n, const BkShape& k) {
  return BkLds(n, 1u << k.hs_log2, k.nch, 0, k.nt / 64).bytes + BK_STATIC_LDS;
}

bool sssp_bucket_fits(uint32_t n) {
  if (n == 0 || (uint64_t)n * 8 >= (1ull << 31)) return false;
  return bk_fixed_lds(n, bk_shape()) <= 160 * 1024;
}

static void launch_sssp_band(sg_ctx* ctx, sg_net* net, BkArgs a, uint32_t n_used, uint32_t rows);

void launch_sssp_bucket(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used, uint32_t row_begin,
                        uint32_t row_end, uint64_t* out_lat, float* out_loss, uint32_t* sat_row,
                        unsigned long long* work, unsigned long long* diag) {
  const uint32_t n = net->n_nodes, rows = row_end - row_begin;
  if (!sssp_bucket_fits(n)) throw Error(SG_ERR_INVALID_ARG, "graph too large for the bucketed search");
  if ((uint64_t)net->n_arcs * 12 >= (1ull << 31)) throw Error(SG_ERR_INVALID_ARG, "too many arcs for 32-bit offsets");
  if (!rows) return;
  hipStream_t st = ctx->stream;
  const BkShape k = bk_shape();
  BkArgs a{};
  a.out_off = net->out_off;
  a.out_arc = net->out_arc;
  a.n = n;
  a.n_arcs = net->n_arcs;
  a.used = d_used;
  a.n_used = n_used;
  a.row_begin = row_begin;
  a.rows = rows;
  a.self_edge = net->self_edge;
  a.e_lat = net->e_lat;
  a.e_loss = net->e_loss;
  a.out_lat = out_lat;
  a.out_loss = out_loss;
  a.sat_row = sat_row;
  // Bucket width: the smallest arc latency, so that a band never relaxes into itself (one pass
  // over its nodes, no re-queued node); where that is tiny next to the arcs' mean (1-ns arcs
  // beside millisecond ones), mean / 128, and the band relaxes its own arcs through the queue.
  // SG_BUCKET_DELTA (ns) overrides.  C5 (w_min 1 ms, mean 50 ms): 1-ms bands, ~270 per row.
  double dl = std::max<double>(std::max<uint32_t>(net->arc_lat_min, 1u), net->arc_lat_mean / 128.0);
  const char* ds = getenv("SG_BUCKET_DELTA");
  if (ds && *ds) dl = atof(ds);
  a.delta = (uint32_t)std::max(1.0, std::min(4294967295.0, dl));
  a.dmul = (uint32_t)(0xFFFFFFFFull / a.delta);
  // ring slots: a power of two <= BK_R (SG_BUCKET_RING; tests: small rings use the far lists)
  const char* rs = getenv("SG_BUCKET_RING");
  uint32_t ring = BK_R;
  if (rs && *rs) {
    ring = 2;
    while (ring < BK_R && ring < (uint32_t)std::max(2, atoi(rs))) ring <<= 1;
  }
  a.ring = ring;
  const char* sm = getenv("SG_SSSP_SPIN_MAX");
  a.spin_max = sm && *sm ? (uint32_t)std::max(1, atoi(sm)) : (1u << 22);
  a.vec_out = n_used % 4 == 0 && ((uintptr_t)out_lat & 15) == 0 && ((uintptr_t)out_loss & 15) == 0;
  a.work = work;
  a.diag = diag;
  // Bands no wider than the smallest arc (the default width wherever that is at least mean / 128):
  // the exact-band kernel; SG_BUCKET_MODE=queue forces the general one
  const char* md = getenv("SG_BUCKET_MODE");
  if (a.delta <= std::max<uint32_t>(net->arc_lat_min, 1u) && !(md && strcmp(md, "queue") == 0)) {
    launch_sssp_band(ctx, net, a, n_used, rows);
    return;
  }
  a.hs_log2 = k.hs_log2;
  a.nch = k.nch;
  // workgroups per CU by the LDS (at most 32 waves per CU), then the entries each can stage in
  // what is left, at most 8192 (SG_BUCKET_STAGE lowers it; tests: 0 stores every entry straight
  // to the arena, small values overflow to it)
  const size_t fixed = bk_fixed_lds(n, k);
  const uint32_t per_cu = (uint32_t)std::max<size_t>(1, std::min<size_t>(std::min<size_t>(
      (size_t)bk_env("SG_BUCKET_PER_CU", 8), 32 / (k.nt / 64)), (160 * 1024) / fixed));
  {
    uint32_t cap = (uint32_t)std::min<size_t>(8192, ((160 * 1024) / per_cu - fixed) / 16);
    const char* sg = getenv("SG_BUCKET_STAGE");
    if (sg && *sg) cap = std::min<uint32_t>(cap, (uint32_t)std::max(0, atoi(sg)));
    a.stg_cap = cap;
  }
  const uint32_t grid = (uint32_t)ctx->n_cu * per_cu;
  uint32_t* ctr = ctx->r_items.get<uint32_t>(2);
  SG_HIP(hipMemsetAsync(ctr, 0, 8, st));
  const size_t arena_b = (size_t)grid * a.nch * BK_CH * 12, scr_b = (size_t)grid * n * 8;
  char* wsp = ctx->r_bucket.get<char>(arena_b + scr_b);
  a.arena = (uint32_t*)wsp;
  a.scratch = (unsigned long long*)(wsp + arena_b);
  a.item_ctr = ctr;
  const size_t lds = BkLds(n, 1u << a.hs_log2, a.nch, a.stg_cap, k.nt / 64).bytes;
  auto go = [&](auto kern, uint32_t nt) {
    SG_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(160 * 1024 - BK_STATIC_LDS)));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(nt), lds, st, a);
  };
  if (k.nt == 1024) {
    if (work) go(k_sssp_bucket<true, 1024, 8>, 1024);
    else go(k_sssp_bucket<false, 1024, 8>, 1024);
  } else {
    if (work) go(k_sssp_bucket<true, 256, 16>, 256);
    else go(k_sssp_bucket<false, 256, 16>, 256);
  }
  SG_CHECK_LAUNCH();
}

// Exact bands (k_sssp_band): bands no wider than the smallest arc latency.
static void launch_sssp_band(sg_ctx* ctx, sg_net* net, BkArgs a, uint32_t n_used, uint32_t rows) {
  hipStream_t st = ctx->stream;
  const uint32_t n = net->n_nodes;
  a.hs_log2 = (uint32_t)std::max(6, std::min(14, bk_env("SG_BUCKET_HASH", 11)));
  a.nch = (uint32_t)std::max(4, std::min(65534, bk_env("SG_BUCKET_CHUNKS", 384)));
  // per-slot staging of the band's appends: off by default -- it coalesces the entry stores but
  // measured slower at C5 (8,192 rows: 47.5 ms with 8 entries per slot, 64.2 ms with 16 (three
  // rows per CU), 45.8 ms without; profiles/r05/ab_band_stage.txt): the kernel is bound by the
  // texture-address unit's lane accesses, not by write requests
  a.stg_cap = (uint32_t)std::max(0, std::min((int)BD_E_MAX, bk_env("SG_BUCKET_STAGE", 0)));
  // band nodes per wave: about 448 arcs, so that a wave's arcs nearly always fit one step of
  // BD_K x 64 slots (C5, mean out-degree 8: 56 nodes, 59.8 against 61.2 ms at 64 for 12,800
  // rows; 48: 60.8, 40: 62.7; profiles/r05/ab_c5_band_npw_r8g.txt); SG_BAND_NPW overrides
  const double mdeg = (double)net->n_arcs / std::max(1u, n);
  a.npw = (uint32_t)std::max(1, std::min(64, bk_env("SG_BAND_NPW", (int)std::max(16.0, std::min(64.0, 448.0 / std::max(mdeg, 1.0))))));
  const size_t lds = BdLds(n, 1u << a.hs_log2, a.nch, 4, a.stg_cap).bytes;
  if (lds + 256 > 160 * 1024) throw Error(SG_ERR_INVALID_ARG, "graph too large for the banded search");
  const uint32_t per_cu = (uint32_t)std::max<size_t>(1, std::min<size_t>((size_t)bk_env("SG_BUCKET_PER_CU", 8),
                                                                         (160 * 1024) / (lds + 256)));
  const uint32_t grid = (uint32_t)ctx->n_cu * per_cu;
  // the graph in the degree-class numbering: built once per sg_net (the workspace remembers its
  // owner, as sg_dense.hip's sorted arcs); the used list mapped every build
  {
    const size_t arc_w = (size_t)net->n_arcs * 3, words = arc_w + 3 * ((size_t)n + 1) + 2 * BD_NCLS + n_used;
    const bool fresh = ctx->band_owner != net->serial || ctx->r_band.cap < words * 4;
    uint32_t* w = ctx->r_band.get<uint32_t>(words);
    uint32_t* barc = w;
    uint32_t* perm = barc + arc_w;
    uint32_t* nbase = perm + n + 1;
    uint32_t* hi = nbase + n + 1;
    uint32_t* cls = hi + n + 1;
    uint32_t* ukey = cls + 2 * BD_NCLS;
    if (fresh) {
      ctx->band_owner = 0;
      TimedLaunch tl(ctx, "band_classes", 0.0);
      hipLaunchKernelGGL(k_band_classes, dim3(1), dim3(BC_T), 0, st, net->out_off, n, perm, nbase, hi, cls);
      hipLaunchKernelGGL(k_band_arcs, dim3(grid_for(n, 256, 4096)), dim3(256), 0, st, net->out_off, net->out_arc, n,
                         perm, nbase, barc);
      SG_CHECK_LAUNCH();
      ctx->band_owner = net->serial;
    }
    hipLaunchKernelGGL(k_band_used, dim3(grid_for(std::max(n_used, 1u), 256, 1024)), dim3(256), 0, st, a.used, n_used,
                       perm, ukey);
    a.out_arc = barc;
    a.hi_off = hi;
    a.cls = cls;
    a.used_key = ukey;
  }
  uint32_t* ctr = ctx->r_items.get<uint32_t>(2);
  SG_HIP(hipMemsetAsync(ctr, 0, 8, st));
  // per-workgroup strides (skewing them by 4-33 KB measured the same, r8d)
  a.arena_words = a.nch * BD_CH * 3;
  a.scr_stride = n;
  // The append filter (SG_BAND_FILTER=1; off by default): n bytes per workgroup, 256-B aligned.
  // Measured at C5 (r6, tools/apsp_ab.py, tables identical; profiles/r06/ab_c5_band_filter_r6d.txt):
  // arena entries 3.98 -> 1.80 per cell, but 287 against 226.5 ms per build -- each filter read is
  // one more dependent L2 / Infinity-Cache round trip on the relaxation's chain (the relax step per
  // band 20.5k -> 34.1k cycles), while the load step it shortens gained only 1.2k (10.8k -> 9.6k):
  // the kernel is bound by the requests each CU keeps in flight (TCP_PENDING_STALL_CYCLES ~0.8 of
  // its cycles, profiles/r05/pmc_band_r06h.txt), and the filter adds a read per live candidate
  const bool filt = bk_env("SG_BAND_FILTER", 0) != 0;
  a.filt_stride = filt ? (n + 255u) / 256u * 256u : 0u;
  const size_t arena_b = ((size_t)grid * a.arena_words * 4 + 255) / 256 * 256, scr_b = (size_t)grid * a.scr_stride * 8;
  const size_t filt_b = (size_t)grid * a.filt_stride;
  char* wsp = ctx->r_bucket.get<char>(arena_b + scr_b + filt_b);
  a.arena = (uint32_t*)wsp;
  a.scratch = (unsigned long long*)(wsp + arena_b);
  a.filt = filt ? (uint8_t*)(wsp + arena_b + scr_b) : nullptr;
  a.item_ctr = ctr;
  (void)rows;
  auto go = [&](auto kern) {
    SG_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, a);
  };
  if (a.work) go(k_sssp_band<true, 256>);
  else go(k_sssp_band<false, 256>);
  SG_CHECK_LAUNCH();
}

}  // namespace sg
