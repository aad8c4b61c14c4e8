// sg_codel.hip -- the routers' inbound CoDel queues, one per host, on the device.
//
// Router::inbound_packets (router/mod.rs:15-58) is a CoDelQueue
// (router/codel_queue.rs): RFC 8289 with Shadow's TARGET = 10 ms and
// INTERVAL = 100 ms, no LIMIT, "good state" while at most one MTU (1500 B,
// definitions.h:124) is stored.  A host's queue is a sequential state machine,
// but hosts are independent: a batch of push / pop events runs one lane per
// host, k_walk-style -- a block owns 64 consecutive hosts, whose events are one
// contiguous range staged through LDS in chunks (coalesced loads, per-host
// sequential processing, coalesced pop results).  The FIFO of each host is a
// ring of `cap` slots in HBM (packet id, enqueue time, length); the scalar
// CoDel state is kept in registers for the whole call.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sg_device.h"
#include "sg_internal.h"

struct sg_codel {
  sg_ctx* ctx = nullptr;
  uint32_t n = 0, cap = 0;
  uint8_t* flags = nullptr;
  uint64_t *iend = nullptr, *dnext = nullptr, *cur = nullptr, *prev = nullptr, *bytes = nullptr;
  uint32_t *head = nullptr, *tail = nullptr;
  uint4* ring = nullptr;  // per slot {packet, len, time lo, time hi}: one 16-B access per push / pop
  unsigned long long* ret = nullptr;  // pinned host-mapped: [dropped, error flags]
  ~sg_codel() {
    void* ps[] = {flags, iend, dnext, cur, prev, bytes, head, tail, ring};
    for (void* p : ps)
      if (p) (void)hipFree(p);
    if (ret) (void)hipHostFree(ret);
  }
};

namespace sg {
namespace {

constexpr uint64_t CD_TARGET = 10000000ull;     // codel_queue.rs:23
constexpr uint64_t CD_INTERVAL = 100000000ull;  // codel_queue.rs:28
constexpr uint64_t CD_MTU = 1500ull;            // definitions.h:124
constexpr uint64_t EMU_MAX = ~0ull - 1;         // emulated_time.rs:30 EMUTIME_MAX
constexpr uint32_t CD_NONE = ~0u;
enum : uint8_t { F_DROP = 1, F_IEND = 2, F_DNEXT = 4 };
enum : uint32_t { E_UNSORTED = 1, E_HOST = 2, E_FULL = 16, E_PKT = 32, E_WINDOW = 64 };

__device__ __forceinline__ uint64_t sat_add(uint64_t t, uint64_t d) { return t > EMU_MAX - d ? EMU_MAX : t + d; }
__device__ __forceinline__ uint64_t since(uint64_t now, uint64_t t) { return now > t ? now - t : 0; }

// apply_control_law (codel_queue.rs:285-298): time + round(INTERVAL / sqrt(count)), f64
__device__ __forceinline__ uint64_t control_law(uint64_t t, uint64_t count) {
  const double s = count == 0 ? 1.0 : sqrt((double)count);
  return sat_add(t, (uint64_t)round((double)CD_INTERVAL / s));
}

// One host's queue (registers) + its ring (HBM).  The head element is also
// cached in registers (hp/ht/hl, valid while head < tail): a pop consumes the
// cache and issues the load of the next element right away, so its latency
// hides behind the events in between instead of stalling the next pop.
// LDS views (address space 3: ds_* instructions, not flat ones)
typedef __attribute__((address_space(3))) const uint32_t lds_u32;
typedef __attribute__((address_space(3))) const uint64_t lds_u64;
typedef __attribute__((address_space(3))) const uint16_t lds_u16;

// s_waitcnt vmcnt(0) as the immediate of __builtin_amdgcn_s_waitcnt (gfx9: lgkmcnt and expcnt
// left at their maxima)
constexpr int VMCNT0 = 0x0F70;

// PF: the kernel keeps the next chunk's loads in flight during the walk (k_codel<LM != 0>); the
// ring path then waits for its own load where it issues it -- where the ring and window paths
// join, the compiler otherwise waits for every vector-memory operation in flight (vmcnt(0)), the
// next chunk's loads included
// ORD (k_inbound<LM, true>, sg_inbound_run_ordered): an element pushed by this call carries
// ARR_BIT | its arrival index instead of the caller's packet id, and its fate is written at that
// index (arrival order: a host's outputs are consecutive) instead of at the packet id.  That is
// unambiguous because no packet id reaches a ring with the bit set: packet ids are below
// n_packets <= 2^31 (the host checks), an id at or past n_packets is refused when it is pushed
// (E_PKT) by the by-id call and when it would be left queued by the ordered one, and an index is
// checked against the call's arrivals before a fate is written at it (after a failed call, e.g.
// a ring overflow, the queue state is undefined but no write leaves the outputs)
constexpr uint32_t ARR_BIT = 0x80000000u;

template <bool PF = false, bool ORD = false>
struct Q {
  uint8_t flags;
  uint64_t iend, dnext, cur, prev, bytes;
  uint32_t head, tail;
  uint32_t hp, hl;
  uint64_t ht;
  bool hv;            // hp/hl/ht hold the element at head
  uint32_t last_len;  // length of the element pop_front returned last
  uint4* ring;
  uint32_t mask;
  // Staged window: the elements this host pushed since begin_window() are the
  // push events of its staged range, in order, so the head element is read
  // from LDS there instead of from the ring in HBM (the ring is still written:
  // what is left at the end of the window lives on in HBM).
  bool win;
  uint32_t t0, wb;  // tail at window start; host's first staged event
  lds_u32 *wp, *wl;
  lds_u64* wt;
  lds_u16* wi;  // the staged index of the window's j-th push, or null: every event is a push
  __device__ void begin_window(lds_u32* p, lds_u32* l, lds_u64* t, lds_u16* pi, uint32_t first) {
    win = true;
    t0 = tail;
    wb = first;
    wp = p;
    wl = l;
    wt = t;
    wi = pi;
  }
  uint8_t* status;
  uint32_t n_status;
  uint64_t dropped;
  uint32_t err;
  uint8_t* astat;  // ORD: per arrival of this call
  uint64_t* afwd;
  uint32_t n_arr;  // ORD: the call's arrivals (the bound of astat / afwd)

  __device__ void drop(uint32_t pkt) {  // drop_packet -> RouterDropped
    if constexpr (ORD) {
      if (pkt & ARR_BIT) {
        if ((pkt & ~ARR_BIT) < n_arr) astat[pkt & ~ARR_BIT] = SG_CODEL_DROPPED;
        else err |= E_PKT;
        dropped++;
        return;
      }
    }
    if (pkt < n_status) status[pkt] = SG_CODEL_DROPPED;
    else err |= E_PKT;
    dropped++;
  }
  // process_standing_delay (codel_queue.rs:231-262)
  __device__ bool standing(uint64_t now, uint64_t sd) {
    if (sd < CD_TARGET || bytes <= CD_MTU) {
      flags &= (uint8_t)~F_IEND;
      return false;
    }
    if (flags & F_IEND) return now >= iend;
    iend = sat_add(now, CD_INTERVAL);
    flags |= F_IEND;
    return false;
  }
  // codel_pop / dodequeue (codel_queue.rs:204-227)
  __device__ bool pop_front(uint64_t now, uint32_t& pkt, bool& ok) {
    if (head == tail) {
      flags &= (uint8_t)~F_IEND;
      return false;
    }
    pkt = hp;
    last_len = hl;
    const uint64_t len = hl, ts = ht;
    head++;
    load_head();
    bytes = bytes > len ? bytes - len : 0;
    ok = standing(now, since(now, ts));
    return true;
  }
  __device__ void load_head() {
    hv = head != tail;
    if (!hv) return;
    const uint32_t j = head - t0;  // the j-th push of the window (modular)
    if (win && j < tail - t0) {
      const uint32_t k = wi ? wi[j] : wb + j;
      hp = wp[k];
      hl = wl[k];
      ht = wt[k];
      return;
    }
    const uint32_t slot = head & mask;
    const uint4 r = ring[slot];
    if constexpr (PF) __builtin_amdgcn_s_waitcnt(VMCNT0);
    hp = r.x;
    hl = r.y;
    ht = ((uint64_t)r.w << 32) | r.z;
  }
  static constexpr bool ord = ORD;
  __device__ bool should_drop(uint64_t now) const { return (flags & F_DNEXT) && now >= dnext; }
  __device__ bool dropping_recently(uint64_t now) const {
    return (flags & F_DNEXT) && since(now, dnext) < 16 * CD_INTERVAL;
  }
  // pop (codel_queue.rs:125-148), drop_from_store_mode (:150-170), drop_from_drop_mode (:172-201)
  __device__ uint32_t pop(uint64_t now) {
    uint32_t pkt;
    bool ok;
    if (!pop_front(now, pkt, ok)) {
      flags &= (uint8_t)~F_DROP;
      return CD_NONE;
    }
    if (!ok) {
      flags &= (uint8_t)~F_DROP;
      return pkt;
    }
    if (!(flags & F_DROP)) {
      drop(pkt);
      uint32_t nxt;
      bool nok;
      const bool has = pop_front(now, nxt, nok);
      flags |= F_DROP;
      const uint64_t delta = cur > prev ? cur - prev : 0;
      cur = (dropping_recently(now) && delta > 1) ? delta : 1;
      dnext = control_law(now, cur);
      flags |= F_DNEXT;
      prev = cur;
      return has ? nxt : CD_NONE;
    }
    bool has = true;
    while (has && (flags & F_DROP) && should_drop(now)) {
      drop(pkt);
      cur++;
      has = pop_front(now, pkt, ok);
      if (has && ok)
        dnext = control_law(dnext, cur);
      else
        flags &= (uint8_t)~F_DROP;
    }
    return has ? pkt : CD_NONE;
  }
  // push (codel_queue.rs:303-317); LIMIT is usize::MAX, the ring is the caller's bound
  __device__ void push(uint32_t pkt, uint64_t now, uint32_t len) {
    if (tail - head > mask) {
      err |= E_FULL;
      return;
    }
    const uint32_t slot = tail & mask;
    ring[slot] = make_uint4(pkt, len, (uint32_t)now, (uint32_t)(now >> 32));
    if (head == tail) {  // the new element is the head
      hp = pkt;
      ht = now;
      hl = len;
      hv = true;
    }
    tail++;
    bytes += len;
  }
};

struct CodelArgs {
  const uint32_t* host_off;
  uint32_t H, E;
  const uint8_t* kind;
  const uint64_t* time;
  const uint32_t* pkt;
  const uint32_t* len;
  uint8_t* flags;
  uint64_t *iend, *dnext, *cur, *prev, *bytes;
  uint32_t *head, *tail;
  uint4* ring;
  uint32_t cap;
  uint32_t* pop_result;
  uint8_t* status;
  uint32_t n_status;
  unsigned long long* blk;  // per block: [dropped, error flags]
  unsigned long long* bdiag = nullptr;  // SG_LANE_DIAG: per block [start, end, walk cycles, most events of a lane]
};

// One wave per block: the walkers are the whole block.  The staging loads are
// unrolled (CD_UNROLL per array in flight per lane) so one wave moves a chunk
// in two rounds of latency.  Blocks with idle helper waves held occupancy
// (VGPRs) without walking: at C4 only 1024 of the 1563 blocks were resident,
// and the kernels ran in two rounds (SG_LANE_DIAG).
constexpr int CD_THREADS = 64;
constexpr int CD_UNROLL = 8;
constexpr int CD_HOSTS = 64;
constexpr int CD_CHUNK = 1024;
constexpr int CD_OUT_CHUNK = 896;  // k_outbound: 24 B per send, 21 KB, 7 blocks per CU
static_assert(CD_THREADS == CD_HOSTS, "a block is its walkers");

// Chunk [c0, c1) staged by the block: ld(i, u) loads element i into slot u of
// the lane's registers, st(k, u) stores slot u to LDS index k.  Indices past
// c1 load element c1 - 1 (always valid, unconditional loads: no branch for the
// compiler to drain each load at) and are not stored.
template <typename LD, typename ST>
__device__ __forceinline__ void stage_chunk(uint32_t c0, uint32_t c1, LD&& ld, ST&& st) {
  const uint32_t t = threadIdx.x;
  for (uint32_t base = c0; base < c1; base += CD_THREADS * CD_UNROLL) {
#pragma unroll
    for (int u = 0; u < CD_UNROLL; u++) ld(min(base + u * CD_THREADS + t, c1 - 1), u);
#pragma unroll
    for (int u = 0; u < CD_UNROLL; u++) {
      const uint32_t i = base + u * CD_THREADS + t;
      if (i < c1) st(i - c0, u);
    }
  }
}

// A block's events in chunks of CH LDS positions.  Contiguous: chunk c is the
// block's events [p0 + c CH, ...), the hosts in order -- at C4 (~20 events per
// host) a chunk holds ~50 hosts' events and every lane walks.  With hundreds of
// events per host (C5: ~200) a contiguous chunk holds ~5 hosts: 5 lanes walk
// while 59 wait, and the block's time is the sum of its hosts' chains.
// Lane-major: chunk c holds events [c LK, (c + 1) LK) of every host, host l at
// positions [l LK, l LK + LK) (holes past a host's last event), so all 64 lanes
// walk every chunk and the block's time is its busiest host's chain.  A host's
// events stay contiguous in position order, so k_codel's push / pop ranks by
// ballot work unchanged (a hole counts as a non-push position: the pop slots
// stay disjoint from the push slots).
template <bool LM, uint32_t CH = CD_CHUNK>
struct ChunkMap {
  static constexpr uint32_t LK = CH / CD_THREADS;  // lane-major: events per host per chunk
  uint32_t p0, p1;                       // the block's event range
  const uint32_t *s_hb, *s_hn;           // lane-major: per host, first event and event count (LDS)
  // chunk c exists (a loop test, not a chunk count: a count's division was hoisted above the
  // walkers' state loads, and its wait for p0 / p1 put a round trip in front of them)
  __device__ bool has(uint32_t c, uint32_t max_n) const { return LM ? c * LK < max_n : p0 + c * CH < p1; }
  // chunk c's positions [0, len)
  __device__ uint32_t len(uint32_t c) const { return LM ? CH : min(CH, p1 - p0 - c * CH); }
  // the event at position k of chunk c (a valid index even when !ok: the loads are unconditional)
  __device__ uint32_t event(uint32_t c, uint32_t k, bool& ok) const {
    if (!LM) {
      const uint32_t i = p0 + c * CH + k;
      ok = i < p1;
      return ok ? i : p1 - 1;
    }
    const uint32_t l = k / LK, o = c * LK + (k % LK), hn = s_hn[l];
    ok = o < hn;
    return ok ? s_hb[l] + o : p0;
  }
  // host lane t's positions [kb, ke) in chunk c, given its events [hb, he); ib = the event at kb
  __device__ void host_range(uint32_t c, uint32_t t, uint32_t hb, uint32_t he, uint32_t& kb, uint32_t& ke,
                             uint32_t& ib) const {
    if (LM) {
      const uint32_t o = c * LK, n = he - hb;
      kb = t * LK;
      ke = kb + (n > o ? min(LK, n - o) : 0u);
      ib = hb + o;
    } else {
      const uint32_t c0 = p0 + c * CH, c1 = min(c0 + CH, p1);
      const uint32_t b = max(hb, c0), e = min(he, c1);
      kb = b < e ? b - c0 : 0;
      ke = b < e ? e - c0 : 0;
      ib = b;
    }
  }
};

// Lane-major when it walks the block in less estimated time: a chunk costs CHUNK_COST walk
// steps of staging and barriers, plus its walk -- contiguous, about one host's share of the
// chunk (the active hosts' mean, capped at CH: its hosts are walked side by side); lane-major,
// LK steps (every host's next LK events side by side).  C5: 13 contiguous chunks of ~200 steps
// against 18 lane-major ones of 16; a partial last block (32 hosts) the same.  A block that is
// mostly one host (5,000 of its 5,006 events) stays contiguous: 313 lane-major chunks.  r05q:
// the earlier rule (lane-major chunks at most twice the contiguous ones) kept the partial last
// block of the C5 round contiguous, and it set every lane kernel's time (k_outbound 592 us walk
// against a 256 us mean).
constexpr uint32_t CHUNK_COST = 10;
template <uint32_t CH = CD_CHUNK>
__device__ __forceinline__ bool lane_major_block(int mode, uint32_t n_ev, uint32_t max_n, uint32_t h_act) {
  if (mode != 2) return mode == 1;
  constexpr uint32_t LK = CH / CD_THREADS;
  if (n_ev <= 2u * CH) return false;  // C4-like blocks: one or two contiguous chunks
  const uint32_t mean = n_ev / max(h_act, 1u);
  const uint64_t c_cost = (uint64_t)((n_ev + CH - 1) / CH) * (CHUNK_COST + min(mean, CH));
  const uint64_t l_cost = (uint64_t)((max_n + LK - 1) / LK) * (CHUNK_COST + LK);
  return l_cost < c_cost;
}

template <bool ANY>
__device__ __forceinline__ uint32_t lane_major_setup(uint32_t hb, uint32_t hn, uint32_t* s_hb, uint32_t* s_hn,
                                                     uint32_t& h_act) {
  if constexpr (!ANY) {
    h_act = 0;
    return 0;
  } else {
    uint32_t max_n = hn;
    for (int o = 32; o > 0; o >>= 1) max_n = max(max_n, (uint32_t)__shfl_xor(max_n, o, 64));
    h_act = (uint32_t)__popcll(__ballot(hn > 0));  // hosts with events in this call
    s_hb[threadIdx.x] = hb;
    s_hn[threadIdx.x] = hn;
    __syncthreads();
    return max_n;
  }
}

// Runs body(ChunkMap<LM, CH>) with the block's layout as a compile-time choice (the
// contiguous path keeps its r04 code; a runtime flag cost C4 ~1.5 us per launch)
// ANY: the kernel was launched with lane-major blocks possible (lane_major_launch).  The
// kernels launched without it keep the r04 contiguous loop verbatim instead of this one:
// walking through ChunkMap<false> cost C4 5-7 % more walk time (k_inbound 22.2 -> 23.5 us
// busiest-lane mean, k_outbound 15.0 -> 16.1, same box, SG_LANE_DIAG)
template <bool ANY, uint32_t CH = CD_CHUNK, class F>
__device__ __forceinline__ void with_chunk_map(bool lm, uint32_t p0, uint32_t p1, const uint32_t* s_hb,
                                               const uint32_t* s_hn, F&& body) {
  if constexpr (ANY) {
    if (lm) {
      body(ChunkMap<true, CH>{p0, p1, s_hb, s_hn});
      return;
    }
  }
  body(ChunkMap<false, CH>{p0, p1, s_hb, s_hn});
}

// SG_LANE_DIAG: a block's start and end on the 100 MHz wall clock (comparable
// across CUs), the cycles its walkers spent walking, and its busiest lane's events
__device__ __forceinline__ void lane_diag_store(unsigned long long* d, uint64_t t0, uint64_t walk, uint32_t ev) {
  if (!d) return;
  if (threadIdx.x < 64) {
    for (int o = 32; o > 0; o >>= 1) {
      walk = max(walk, (uint64_t)__shfl_xor((unsigned long long)walk, o, 64));
      ev = max(ev, (uint32_t)__shfl_xor(ev, o, 64));
    }
    if (threadIdx.x == 0) {
      unsigned long long* q = d + 4 * (size_t)blockIdx.x;
      q[0] = t0;
      q[1] = wall_clock64();
      q[2] = walk;
      q[3] = ev;
    }
  }
}

// LM: the chunk layouts this launch may use (lane_major_launch): 0 contiguous only, 1 lane-major
// only, 2 per block (lane_major_block).  A template parameter, not an argument: a field added to
// the argument structs changed k_inbound's register allocation and cost C4 ~2 us.
template <int LM>
__global__ void __launch_bounds__(CD_THREADS) k_codel(CodelArgs a) {
  constexpr bool ANY = LM != 0;
  const uint64_t d_t0 = a.bdiag ? wall_clock64() : 0;
  uint64_t d_walk = 0;
  // Staged chunk, 18 KB (8 one-wave blocks fit a CU): the chunk's pushes in push order
  // from the front of s_t / s_p / s_l (time, packet, length), its pops in pop order from
  // the back (time, result, pushes before the pop), so a walk step reads its element and
  // its next pop's fields directly -- no index list between (r03: an index read, then the
  // data, at every pop and every push accounted)
  __shared__ uint64_t s_t[CD_CHUNK];
  __shared__ uint32_t s_p[CD_CHUNK];
  __shared__ uint32_t s_l[CD_CHUNK];
  __shared__ uint16_t s_pp[CD_CHUNK + 1];  // pushes before each staged event (kind k = s_pp[k + 1] - s_pp[k])
  auto pop_at = [](uint32_t r) { return (uint32_t)CD_CHUNK - 1u - r; };  // the r-th pop's slot
  const uint32_t h0 = blockIdx.x * CD_HOSTS, t = threadIdx.x;
  const uint32_t p0 = min(a.host_off[min(h0, a.H)], a.E);
  const uint32_t p1 = max(min(a.host_off[min(h0 + CD_HOSTS, a.H)], a.E), p0);
  const uint32_t h = h0 + t;
  const bool walker = t < CD_HOSTS && h < a.H;
  uint32_t hb = 0, he = 0;
  Q<LM != 0> q{};
  if (walker) {
    hb = min(a.host_off[h], a.E);
    he = max(min(a.host_off[h + 1], a.E), hb);
    q.flags = a.flags[h];
    q.iend = a.iend[h];
    q.dnext = a.dnext[h];
    q.cur = a.cur[h];
    q.prev = a.prev[h];
    q.bytes = a.bytes[h];
    q.head = a.head[h];
    q.tail = a.tail[h];
    q.ring = a.ring + (size_t)h * a.cap;
    q.mask = a.cap - 1;
    q.status = a.status;
    q.n_status = a.n_status;
    q.load_head();
  }
  const uint64_t lt = (1ull << t) - 1;  // lanes below this one
  if constexpr (!ANY) {  // contiguous chunks only: the r04 loop as it was (see with_chunk_map)
  for (uint32_t c0 = p0; c0 < p1; c0 += CD_CHUNK) {
    const uint32_t c1 = min(c0 + CD_CHUNK, p1);
    {  // 1. coalesced staging, and the chunk's push and pop lists by ballot (the block is one wave)
      uint32_t run = 0;
      for (uint32_t base = c0; base < c1; base += CD_THREADS * CD_UNROLL) {
        uint64_t rt[CD_UNROLL];
        uint32_t rp[CD_UNROLL], rl[CD_UNROLL];
        uint8_t rk[CD_UNROLL];
#pragma unroll
        for (int u = 0; u < CD_UNROLL; u++) {
          const uint32_t i = min(base + u * CD_THREADS + t, c1 - 1);
          rt[u] = a.time[i];
          rp[u] = a.pkt[i];
          rl[u] = a.len[i];
          rk[u] = a.kind[i];
        }
#pragma unroll
        for (int u = 0; u < CD_UNROLL; u++) {
          const uint32_t i = base + u * CD_THREADS + t;
          const bool in = i < c1, push = in && rk[u] == SG_CODEL_PUSH;
          const uint64_t m = __ballot(push);
          const uint32_t rank = run + (uint32_t)__popcll(m & lt);
          if (in) {
            const uint32_t k = i - c0;
            const uint32_t slot = push ? rank : pop_at(k - rank);
            s_t[slot] = rt[u];
            s_p[slot] = rp[u];
            s_l[slot] = push ? rl[u] : rank;
            s_pp[k] = (uint16_t)rank;
          }
          run += (uint32_t)__popcll(m);
        }
      }
      if (t == 0) s_pp[c1 - c0] = (uint16_t)run;
    }
    __syncthreads();
    if (walker) {
      // 2. each host's pops in order.  A host's pushes between two pops only
      // append (tail, bytes): they are accounted at the next pop, the elements
      // read from the staged window, and the ring is written at the chunk's end
      // for the elements still queued -- the walk's steps are the pops alone.
      const uint64_t d_w0 = a.bdiag ? clock64() : 0;
      // this host's staged range [kb, ke) (empty when its events lie outside the chunk)
      const uint32_t b = max(hb, c0), e = min(he, c1);
      const uint32_t kb = b < e ? b - c0 : 0, ke = b < e ? e - c0 : 0;
      const uint32_t pb = kb < ke ? s_pp[kb] : 0, pe = kb < ke ? s_pp[ke] : 0;
      const uint32_t rb = kb - pb, re = ke - pe;  // this host's pop ranks [rb, re)
      // the window's j-th push is push slot pb + j
      q.begin_window((lds_u32*)s_p, (lds_u32*)s_l, (lds_u64*)s_t, nullptr, pb);
      uint32_t seen = 0;  // window pushes accounted
      auto account = [&](uint32_t upto) {  // the window's pushes [seen, upto) enter the queue
        for (; seen < upto; seen++) q.bytes += s_l[pb + seen];
        q.tail = q.t0 + upto;
        if (q.tail - q.head > q.mask + 1u) q.err |= E_FULL;  // a push found the ring full
        if (!q.hv) q.load_head();
      };
      // the next pop's fields are read a step ahead
      uint64_t t1 = rb < re ? s_t[pop_at(rb)] : 0;
      uint32_t pp1 = rb < re ? s_l[pop_at(rb)] : 0;
      for (uint32_t r = rb; r < re; r++) {
        const uint32_t k = pop_at(r), pp = pp1;
        const uint64_t now = t1;
        if (r + 1 < re) {
          t1 = s_t[pop_at(r + 1)];
          pp1 = s_l[pop_at(r + 1)];
        }
        account(pp - pb);
        const uint32_t res = q.pop(now);
        // a dequeued packet's status is written with the chunk's results (3. below): a
        // global store here made the walk's next vector-memory wait (the ring prefetch,
        // or a register the compiler shares with it) wait for the store too
        if (res != CD_NONE && res >= q.n_status) q.err |= E_PKT;
        s_p[k] = res;  // a pop's packet slot is read by no one else
      }
      account(pe - pb);
      // the window's elements still queued live on in the ring
      const uint32_t w0 = q.head - q.t0 <= q.tail - q.t0 ? q.head - q.t0 : 0;
      for (uint32_t j = w0; j < q.tail - q.t0; j++) {
        const uint32_t k = pb + j;
        const uint64_t tk = s_t[k];
        q.ring[(q.t0 + j) & q.mask] = make_uint4(s_p[k], s_l[k], (uint32_t)tk, (uint32_t)(tk >> 32));
      }
      if (a.bdiag) d_walk += clock64() - d_w0;
      q.win = false;  // the next chunk's staging overwrites the window (the head stays cached)
    }
    __syncthreads();
    for (uint32_t i = c0 + t; i < c1; i += CD_THREADS) {  // 3. coalesced results (CD_NONE for a push)
      const uint32_t k = i - c0;
      const uint32_t r = s_pp[k + 1] != s_pp[k] ? CD_NONE : s_p[pop_at(k - s_pp[k])];
      a.pop_result[i] = r;
      if (r < a.n_status) a.status[r] = SG_CODEL_DEQUEUED;  // (CD_NONE >= n_status)
    }
    __syncthreads();
  }
  } else {
  __shared__ uint32_t s_hb[CD_HOSTS], s_hn[CD_HOSTS];
  const uint32_t hn = he - hb;
  uint32_t h_act;
  const uint32_t max_n = lane_major_setup<ANY>(hb, hn, s_hb, s_hn, h_act);
  with_chunk_map<ANY>(ANY && lane_major_block(LM, p1 - p0, max_n, h_act), p0, p1, s_hb, s_hn, [&](auto cm) {
  // A chunk's events are loaded into registers a chunk ahead (CD_PF per lane, one round of
  // loads): the next chunk's loads are in flight during this chunk's walk.  At C5 a block walks
  // ~19 lane-major chunks, and each chunk's staging round trips sat in front of its walk.
  constexpr int CD_PF = CD_CHUNK / CD_THREADS;
  uint64_t rt[CD_PF];
  uint32_t rp[CD_PF], rl[CD_PF];
  uint8_t rk[CD_PF];
  bool ok[CD_PF];
  auto fetch = [&](uint32_t f) {
#pragma unroll
    for (int u = 0; u < CD_PF; u++) {
      const uint32_t i = cm.event(f, u * CD_THREADS + t, ok[u]);
      rt[u] = a.time[i];
      rp[u] = a.pkt[i];
      rl[u] = a.len[i];
      rk[u] = a.kind[i];
    }
  };
  if (cm.has(0, max_n)) fetch(0);
  for (uint32_t c = 0; cm.has(c, max_n); c++) {
    const uint32_t clen = cm.len(c);
    {  // 1. staging from the registers (the chunk's range, or 16-event runs per host), and the
       //    chunk's push and pop lists by ballot (the block is one wave)
      uint32_t run = 0;
#pragma unroll
      for (int u = 0; u < CD_PF; u++) {
        const uint32_t k = u * CD_THREADS + t;
        const bool in = k < clen, push = in && ok[u] && rk[u] == SG_CODEL_PUSH;
        const uint64_t m = __ballot(push);
        const uint32_t rank = run + (uint32_t)__popcll(m & lt);
        if (in) {
          const uint32_t slot = push ? rank : pop_at(k - rank);
          if (ok[u]) {
            s_t[slot] = rt[u];
            s_p[slot] = rp[u];
            s_l[slot] = push ? rl[u] : rank;
          }
          s_pp[k] = (uint16_t)rank;
        }
        run += (uint32_t)__popcll(m);
      }
      if (t == 0) s_pp[clen] = (uint16_t)run;
    }
    if (cm.has(c + 1, max_n)) fetch(c + 1);  // (uniform) in flight during the walk
    __syncthreads();
    if (walker) {
      // 2. each host's pops in order.  A host's pushes between two pops only
      // append (tail, bytes): they are accounted at the next pop, the elements
      // read from the staged window, and the ring is written at the chunk's end
      // for the elements still queued -- the walk's steps are the pops alone.
      const uint64_t d_w0 = a.bdiag ? clock64() : 0;
      // this host's staged positions [kb, ke) (empty when none of its events is in the chunk)
      uint32_t kb, ke, ib;
      cm.host_range(c, t, hb, he, kb, ke, ib);
      (void)ib;
      const uint32_t pb = kb < ke ? s_pp[kb] : 0, pe = kb < ke ? s_pp[ke] : 0;
      const uint32_t rb = kb - pb, re = ke - pe;  // this host's pop ranks [rb, re)
      // the window's j-th push is push slot pb + j
      q.begin_window((lds_u32*)s_p, (lds_u32*)s_l, (lds_u64*)s_t, nullptr, pb);
      uint32_t seen = 0;  // window pushes accounted
      auto account = [&](uint32_t upto) {  // the window's pushes [seen, upto) enter the queue
        for (; seen < upto; seen++) q.bytes += s_l[pb + seen];
        q.tail = q.t0 + upto;
        if (q.tail - q.head > q.mask + 1u) q.err |= E_FULL;  // a push found the ring full
        if (!q.hv) q.load_head();
      };
      // the next pop's fields are read a step ahead
      uint64_t t1 = rb < re ? s_t[pop_at(rb)] : 0;
      uint32_t pp1 = rb < re ? s_l[pop_at(rb)] : 0;
      for (uint32_t r = rb; r < re; r++) {
        const uint32_t k = pop_at(r), pp = pp1;
        const uint64_t now = t1;
        if (r + 1 < re) {
          t1 = s_t[pop_at(r + 1)];
          pp1 = s_l[pop_at(r + 1)];
        }
        account(pp - pb);
        const uint32_t res = q.pop(now);
        // a dequeued packet's status is written with the chunk's results (3. below): a
        // global store here made the walk's next vector-memory wait (the ring prefetch,
        // or a register the compiler shares with it) wait for the store too
        if (res != CD_NONE && res >= q.n_status) q.err |= E_PKT;
        s_p[k] = res;  // a pop's packet slot is read by no one else
      }
      account(pe - pb);
      // the window's elements still queued live on in the ring
      const uint32_t w0 = q.head - q.t0 <= q.tail - q.t0 ? q.head - q.t0 : 0;
      for (uint32_t j = w0; j < q.tail - q.t0; j++) {
        const uint32_t k = pb + j;
        const uint64_t tk = s_t[k];
        q.ring[(q.t0 + j) & q.mask] = make_uint4(s_p[k], s_l[k], (uint32_t)tk, (uint32_t)(tk >> 32));
      }
      if (a.bdiag) d_walk += clock64() - d_w0;
      q.win = false;  // the next chunk's staging overwrites the window (the head stays cached)
    }
    __syncthreads();
    for (uint32_t k = t; k < clen; k += CD_THREADS) {  // 3. results (CD_NONE for a push)
      bool ok;
      const uint32_t i = cm.event(c, k, ok);
      if (!ok) continue;
      const uint32_t r = s_pp[k + 1] != s_pp[k] ? CD_NONE : s_p[pop_at(k - s_pp[k])];
      a.pop_result[i] = r;
      if (r < a.n_status) a.status[r] = SG_CODEL_DEQUEUED;  // (CD_NONE >= n_status)
    }
    __syncthreads();
  }
  });
  }
  unsigned long long dropped = 0, err = 0;
  if (walker) {
    a.flags[h] = q.flags;
    a.iend[h] = q.iend;
    a.dnext[h] = q.dnext;
    a.cur[h] = q.cur;
    a.prev[h] = q.prev;
    a.bytes[h] = q.bytes;
    a.head[h] = q.head;
    a.tail[h] = q.tail;
    dropped = q.dropped;
    err = q.err;
  }
  lane_diag_store(a.bdiag, d_t0, d_walk, he - hb);
  if (t < 64) {
    for (int d = 32; d > 0; d >>= 1) {
      dropped += __shfl_xor(dropped, d, 64);
      err |= __shfl_xor(err, d, 64);
    }
    if (t == 0) {
      a.blk[2 * blockIdx.x] = dropped;
      a.blk[2 * blockIdx.x + 1] = err;
    }
  }
}

// Sums the blocks' drop counts, ORs their error flags (and the grouping
// check's) into the pinned host-mapped return block.
__global__ void __launch_bounds__(1024) k_codel_reduce(const unsigned long long* __restrict__ blk, uint32_t n,
                                                       const uint32_t* __restrict__ group_err,
                                                       unsigned long long* __restrict__ ret) {
  __shared__ unsigned long long r[2][16];
  unsigned long long d = 0, e = 0;
  for (uint32_t i = threadIdx.x; i < n; i += 1024) {
    d += blk[2 * i];
    e |= blk[2 * i + 1];
  }
  for (int s = 32; s > 0; s >>= 1) {
    d += __shfl_xor(d, s, 64);
    e |= __shfl_xor(e, s, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    r[0][threadIdx.x >> 6] = d;
    r[1][threadIdx.x >> 6] = e;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 16; i++) {
      d += r[0][i];
      e |= r[1][i];
    }
    ret[0] = d;
    ret[1] = e | *group_err;
  }
}

// ---- inbound pipeline: router CoDel queue -> relay_inet_in ---------------
// Per host over a window of simulated time (relay/mod.rs:72-288,
// relay/token_bucket.rs, host.rs:781-786, :919-924): each arrival (a Packet
// event, in EventQueue order) pushes into the host's CoDel queue and notifies
// the inbound relay; an Idle relay schedules its forward task at that time (a
// Local event: after the Packet events of the same time, event.rs:103-112; it
// takes an event id, host.rs:649-653).  The task pops until the queue is empty
// or the token bucket blocks, then reschedules itself after the conforming
// duration.  Tasks at or after the window end stay pending for the next call.
constexpr uint64_t TB_INTERVAL = 1000000ull;  // relay/mod.rs:297: refill every 1 ms
enum : uint8_t { R_PENDING = 1, R_NEVER = 2, R_CACHED = 4 };

struct Relay {
  uint8_t rf;
  uint64_t tt;  // pending task time
  uint32_t cp, cl;  // cached packet, its length
  uint64_t cap, bal, inc, last;  // token bucket (token_bucket.rs:6-12)
  uint64_t n_max;                 // u64::MAX / inc (inc != 0): the refill count past which tokens saturate
  uint64_t ctr0;                  // the host's event counter at the call's start (0 without event_ctr)
  uint64_t tid, tborn;            // the pending task's event id and creation time (Event::new_local)

  // forward_later: the task is a Local event created at `now` (host.rs:690-697); its id is the
  // host counter's next value (host.rs:649-653), taken even when it lands past sim_end
  __device__ void schedule(uint64_t now, uint64_t at, uint64_t sim_end, uint64_t& ctr_inc) {
    rf |= R_PENDING;
    tid = ctr0 + ctr_inc++;
    tborn = now;
    tt = at;
    if (at >= sim_end) rf |= R_NEVER;
  }

  // inc is fixed for the call: the one u64 division by it happens here, not on every refill
  __device__ void set_inc(uint64_t v) {
    inc = v;
    n_max = v ? ~0ull / v : ~0ull;
  }
  // lazy_refill (token_bucket.rs:124-158): the span to the next refill
  __device__ uint64_t lazy_refill(uint64_t now) {
    uint64_t span = now - last;
    if (span >= TB_INTERVAL) {
      const uint64_t n = span / TB_INTERVAL;
      const uint64_t tokens = (inc != 0 && n > n_max) ? ~0ull : inc * n;
      const uint64_t b = bal > ~0ull - tokens ? ~0ull : bal + tokens;
      bal = b > cap ? cap : b;
      last = sat_add(last, n > ~0ull / TB_INTERVAL ? ~0ull : TB_INTERVAL * n);
      span = now - last;
    }
    return TB_INTERVAL - span;
  }
  // conforming_remove (token_bucket.rs:76-118)
  __device__ bool remove(uint64_t dec, uint64_t now, uint64_t& wait) {
    const uint64_t next = lazy_refill(now);
    if (bal >= dec) {
      bal -= dec;
      return true;
    }
    const uint64_t need = dec - bal;
    const uint64_t qn = need / inc;
    const uint64_t nref = qn + (need - qn * inc ? 1 : 0);
    if (nref == 1) {
      wait = next;
    } else {
      const uint64_t m = nref - 1;
      const uint64_t extra = m > ~0ull / TB_INTERVAL ? ~0ull : TB_INTERVAL * m;
      wait = next > ~0ull - extra ? ~0ull : next + extra;
    }
    return false;
  }
};

struct InboundArgs {
  CodelArgs q;  // queues; q.kind unused (every event is an arrival)
  uint8_t* rflags;
  uint64_t* task_time;
  uint32_t *cached_pkt, *cached_len;
  uint64_t *tb_cap, *tb_bal, *tb_inc, *tb_last;
  uint64_t window_end, bootstrap_end, sim_end;
  uint64_t* event_ctr;  // per host, or null
  uint64_t* fwd_time;   // per packet
  uint64_t *task_id, *task_born;  // per host: the pending task's event id and creation time
  uint8_t* arr_status;  // ORD: per arrival
  uint64_t* arr_fwd;
};

// The relay's forward task at `now` (run_forward_task -> forward_until_blocked).
template <class QT>
__device__ void relay_task(QT& q, Relay& r, uint64_t now, uint64_t bootstrap_end, uint64_t sim_end,
                           uint64_t& ctr_inc, uint64_t* fwd_time) {
  r.rf &= (uint8_t)~R_PENDING;
  for (;;) {
    uint32_t p, l;
    if (r.rf & R_CACHED) {
      p = r.cp;
      l = r.cl;
      r.rf &= (uint8_t)~R_CACHED;
    } else {
      const uint32_t popped = q.pop(now);
      if (popped == CD_NONE) return;  // empty: Idle
      p = popped;
      l = q.last_len;  // the popped element is the last one pop_front returned
    }
    uint64_t wait;
    if (now >= bootstrap_end && !r.remove(l, now, wait)) {  // Worker::is_bootstrapping: no rate limit
      r.rf |= R_CACHED;  // RelayCached; forward_later(wait)
      r.cp = p;
      r.cl = l;
      r.schedule(now, now > ~0ull - wait ? ~0ull : now + wait, sim_end, ctr_inc);
      return;
    }
    if (QT::ord && (p & ARR_BIT)) {  // RelayForwarded, an arrival of this call: at its index
      if ((p & ~ARR_BIT) < q.n_arr) {
        q.astat[p & ~ARR_BIT] = SG_CODEL_DEQUEUED;
        q.afwd[p & ~ARR_BIT] = now;
      } else {
        q.err |= E_PKT;
      }
    } else if (p < q.n_status) {  // RelayForwarded: pushed to the internet interface
      q.status[p] = SG_CODEL_DEQUEUED;
      fwd_time[p] = now;
    } else {
      q.err |= E_PKT;
    }
  }
}

template <int LM, bool ORD = false>
__global__ void __launch_bounds__(CD_THREADS) k_inbound(InboundArgs ia) {
  constexpr bool ANY = LM != 0;
  const uint64_t d_t0 = ia.q.bdiag ? wall_clock64() : 0;
  uint64_t d_walk = 0;
  const CodelArgs& a = ia.q;
  __shared__ uint64_t s_t[CD_CHUNK];
  __shared__ uint32_t s_p[CD_CHUNK];
  __shared__ uint32_t s_l[CD_CHUNK];
  const uint32_t h0 = blockIdx.x * CD_HOSTS, t = threadIdx.x;
  const uint32_t p0 = min(a.host_off[min(h0, a.H)], a.E);
  const uint32_t p1 = max(min(a.host_off[min(h0 + CD_HOSTS, a.H)], a.E), p0);
  const uint32_t h = h0 + t;
  const bool walker = t < CD_HOSTS && h < a.H;
  uint32_t hb = 0, he = 0;
  Q<false, ORD> q{};
  Relay r{};
  uint64_t ctr_inc = 0;
  uint32_t tail0 = 0;  // ORD: the tail at the call's start (later elements carry arrival indices)
  bool id_bad = false;  // !ORD: a staged packet id at or past n_packets (refused when it is pushed: E_PKT)
  if (walker) {
    hb = min(a.host_off[h], a.E);
    he = max(min(a.host_off[h + 1], a.E), hb);
    q.flags = a.flags[h];
    q.iend = a.iend[h];
    q.dnext = a.dnext[h];
    q.cur = a.cur[h];
    q.prev = a.prev[h];
    q.bytes = a.bytes[h];
    q.head = a.head[h];
    q.tail = a.tail[h];
    q.ring = a.ring + (size_t)h * a.cap;
    q.mask = a.cap - 1;
    q.status = a.status;
    q.n_status = a.n_status;
    q.astat = ia.arr_status;
    q.afwd = ia.arr_fwd;
    q.n_arr = a.E;
    tail0 = q.tail;
    q.load_head();
    r.rf = ia.rflags[h];
    r.tt = ia.task_time[h];
    r.cp = ia.cached_pkt[h];
    r.cl = ia.cached_len[h];
    r.cap = ia.tb_cap[h];
    r.bal = ia.tb_bal[h];
    r.set_inc(ia.tb_inc[h]);
    r.last = ia.tb_last[h];
    r.ctr0 = ia.event_ctr ? ia.event_ctr[h] : 0;
    r.tid = ia.task_id[h];
    r.tborn = ia.task_born[h];
  }
  auto due = [&](uint64_t before) {  // a pending task earlier than `before` (Packet events go first)
    return (r.rf & R_PENDING) && !(r.rf & R_NEVER) && r.tt < before;
  };
  if constexpr (!ANY) {  // contiguous chunks only: the r04 loop as it was (see with_chunk_map)
  for (uint32_t c0 = p0; c0 < p1; c0 += CD_CHUNK) {
    const uint32_t c1 = min(c0 + CD_CHUNK, p1);
    {
      uint64_t rt[CD_UNROLL];
      uint32_t rp[CD_UNROLL], rl[CD_UNROLL];
      stage_chunk(
          c0, c1,
          [&](uint32_t i, int u) {
            rt[u] = a.time[i];
            rp[u] = ORD ? (ARR_BIT | i) : a.pkt[i];
            if (!ORD) id_bad |= rp[u] >= a.n_status;
            rl[u] = a.len[i];
          },
          [&](uint32_t k, int u) {
            s_t[k] = rt[u];
            s_p[k] = rp[u];
            s_l[k] = rl[u];
          });
    }
    __syncthreads();
    if (walker) {
      const uint32_t b = max(hb, c0), e = min(he, c1);
      const uint64_t d_w0 = a.bdiag ? clock64() : 0;
      q.win = false;  // the tasks first run by this chunk pop the previous chunk's elements from HBM
      q.begin_window((lds_u32*)s_p, (lds_u32*)s_l, (lds_u64*)s_t, nullptr, b - c0);
      uint64_t nt = b < e ? s_t[b - c0] : 0;  // the next arrival's fields, read ahead
      uint32_t np = b < e ? s_p[b - c0] : 0, nl = b < e ? s_l[b - c0] : 0;
      for (uint32_t i = b; i < e; i++) {
        const uint32_t k = i - c0;
        const uint64_t now = nt;
        const uint32_t pkt = np, len = nl;
        if (i + 1 < e) {
          nt = s_t[k + 1];
          np = s_p[k + 1];
          nl = s_l[k + 1];
        }
        if (now >= ia.window_end) q.err |= E_WINDOW;
        while (due(now)) relay_task(q, r, r.tt, ia.bootstrap_end, ia.sim_end, ctr_inc, ia.fwd_time);
        // Router::route_incoming_packet: the arrival is the window's next element (staged
        // slot k, read from LDS when it reaches the head); the ring receives the window's
        // still-queued elements at the chunk's end, as in k_codel -- a ring store per
        // arrival made the walk's next vector-memory wait include it
        (void)pkt;
        q.tail++;
        q.bytes += len;
        if (q.tail - q.head > q.mask + 1u) q.err |= E_FULL;  // an arrival found the ring full
        if (!q.hv) q.load_head();
        if (!(r.rf & R_PENDING)) r.schedule(now, now, ia.sim_end, ctr_inc);  // notify: Idle -> forward_later(ZERO)
      }
      // the window's elements still queued live on in the ring
      const uint32_t w0 = q.head - q.t0 <= q.tail - q.t0 ? q.head - q.t0 : 0;
      for (uint32_t j = w0; j < q.tail - q.t0; j++) {
        const uint32_t k = q.wb + j;
        const uint64_t tk = s_t[k];
        q.ring[(q.t0 + j) & q.mask] = make_uint4(s_p[k], s_l[k], (uint32_t)tk, (uint32_t)(tk >> 32));
      }
      q.win = false;  // the next chunk's staging overwrites the window
      if (a.bdiag) d_walk += clock64() - d_w0;
    }
    __syncthreads();
  }
  } else {
  __shared__ uint32_t s_hb[CD_HOSTS], s_hn[CD_HOSTS];
  uint32_t h_act;
  const uint32_t max_n = lane_major_setup<ANY>(hb, he - hb, s_hb, s_hn, h_act);
  with_chunk_map<ANY>(ANY && lane_major_block(LM, p1 - p0, max_n, h_act), p0, p1, s_hb, s_hn, [&](auto cm) {
  for (uint32_t c = 0; cm.has(c, max_n); c++) {
    const uint32_t clen = cm.len(c);
    for (uint32_t base = 0; base < clen; base += CD_THREADS * CD_UNROLL) {  // staging (see ChunkMap)
      uint64_t rt[CD_UNROLL];
      uint32_t rp[CD_UNROLL], rl[CD_UNROLL];
      bool ok[CD_UNROLL];
#pragma unroll
      for (int u = 0; u < CD_UNROLL; u++) {
        const uint32_t i = cm.event(c, base + u * CD_THREADS + t, ok[u]);
        rt[u] = a.time[i];
        rp[u] = ORD ? (ARR_BIT | i) : a.pkt[i];
        if (!ORD) id_bad |= rp[u] >= a.n_status;
        rl[u] = a.len[i];
      }
#pragma unroll
      for (int u = 0; u < CD_UNROLL; u++) {
        const uint32_t k = base + u * CD_THREADS + t;
        if (k < clen && ok[u]) {
          s_t[k] = rt[u];
          s_p[k] = rp[u];
          s_l[k] = rl[u];
        }
      }
    }
    __syncthreads();
    if (walker) {
      uint32_t kb, ke, ib;
      cm.host_range(c, t, hb, he, kb, ke, ib);
      (void)ib;
      const uint64_t d_w0 = a.bdiag ? clock64() : 0;
      q.win = false;  // the tasks first run by this chunk pop the previous chunk's elements from HBM
      q.begin_window((lds_u32*)s_p, (lds_u32*)s_l, (lds_u64*)s_t, nullptr, kb);
      uint64_t nt = kb < ke ? s_t[kb] : 0;  // the next arrival's fields, read ahead
      uint32_t np = kb < ke ? s_p[kb] : 0, nl = kb < ke ? s_l[kb] : 0;
      for (uint32_t k = kb; k < ke; k++) {
        const uint64_t now = nt;
        const uint32_t pkt = np, len = nl;
        if (k + 1 < ke) {
          nt = s_t[k + 1];
          np = s_p[k + 1];
          nl = s_l[k + 1];
        }
        if (now >= ia.window_end) q.err |= E_WINDOW;
        while (due(now)) relay_task(q, r, r.tt, ia.bootstrap_end, ia.sim_end, ctr_inc, ia.fwd_time);
        // Router::route_incoming_packet: the arrival is the window's next element (staged
        // slot k, read from LDS when it reaches the head); the ring receives the window's
        // still-queued elements at the chunk's end, as in k_codel -- a ring store per
        // arrival made the walk's next vector-memory wait include it
        (void)pkt;
        q.tail++;
        q.bytes += len;
        if (q.tail - q.head > q.mask + 1u) q.err |= E_FULL;  // an arrival found the ring full
        if (!q.hv) q.load_head();
        if (!(r.rf & R_PENDING)) r.schedule(now, now, ia.sim_end, ctr_inc);  // notify: Idle -> forward_later(ZERO)
      }
      // the window's elements still queued live on in the ring
      const uint32_t w0 = q.head - q.t0 <= q.tail - q.t0 ? q.head - q.t0 : 0;
      for (uint32_t j = w0; j < q.tail - q.t0; j++) {
        const uint32_t k = q.wb + j;
        const uint64_t tk = s_t[k];
        q.ring[(q.t0 + j) & q.mask] = make_uint4(s_p[k], s_l[k], (uint32_t)tk, (uint32_t)(tk >> 32));
      }
      q.win = false;  // the next chunk's staging overwrites the window
      if (a.bdiag) d_walk += clock64() - d_w0;
    }
    __syncthreads();
  }
  });
  }
  unsigned long long err = 0, dropped = 0;
  if (walker) {
    while (due(ia.window_end)) relay_task(q, r, r.tt, ia.bootstrap_end, ia.sim_end, ctr_inc, ia.fwd_time);
    if constexpr (ORD) {
      // the elements this call pushed that are still queued (the last min(queued, pushed) of
      // the ring), and a cached one, go back to the caller's packet ids for the next call; an id
      // past n_packets would read as an index in a later call, so it fails this one (E_PKT).
      // After a ring overflow (E_FULL: the call fails with SG_ERR_CAPACITY) the ring no longer
      // holds those elements, and nothing is translated
      auto to_id = [&](uint32_t v) -> uint32_t {
        const uint32_t i = v & ~ARR_BIT;
        const uint32_t id = i < a.E ? a.pkt[i] : 0xFFFFFFFFu;
        if (id >= a.n_status) q.err |= E_PKT;
        return id;
      };
      if (!(q.err & E_FULL)) {
        const uint32_t pushed = q.tail - tail0, queued = q.tail - q.head;
        for (uint32_t j = q.tail - min(min(pushed, queued), q.mask + 1u); j != q.tail; j++) {
          uint32_t* x = (uint32_t*)&q.ring[j & q.mask];
          if (*x & ARR_BIT) *x = to_id(*x);
        }
        if ((r.rf & R_CACHED) && (r.cp & ARR_BIT)) r.cp = to_id(r.cp);
      }
    }
    a.flags[h] = q.flags;
    a.iend[h] = q.iend;
    a.dnext[h] = q.dnext;
    a.cur[h] = q.cur;
    a.prev[h] = q.prev;
    a.bytes[h] = q.bytes;
    a.head[h] = q.head;
    a.tail[h] = q.tail;
    ia.rflags[h] = r.rf;
    ia.task_time[h] = r.tt;
    ia.cached_pkt[h] = r.cp;
    ia.cached_len[h] = r.cl;
    ia.tb_bal[h] = r.bal;
    ia.tb_last[h] = r.last;
    ia.task_id[h] = r.tid;
    ia.task_born[h] = r.tborn;
    if (ia.event_ctr && ctr_inc) ia.event_ctr[h] += ctr_inc;
    err = q.err;
    dropped = q.dropped;
  }
  if (!ORD && id_bad) err |= E_PKT;  // (every lane staged ids)
  lane_diag_store(a.bdiag, d_t0, d_walk, he - hb);
  if (t < 64) {
    for (int d = 32; d > 0; d >>= 1) {
      dropped += __shfl_xor(dropped, d, 64);
      err |= __shfl_xor(err, d, 64);
    }
    if (t == 0) {
      a.blk[2 * blockIdx.x] = dropped;
      a.blk[2 * blockIdx.x + 1] = err;
    }
  }
}

// ---- outbound pipeline: interface FIFO -> relay_inet_out -> router --------
// Per host: sends push {packet, len, dst, payload_len} records into a ring
// (the interface's fifo qdisc); the relay's forward task pops them in order.
// The packet a blocked relay caches is the slot at head - 1 (never
// overwritten: a call's pushes may not reach the oldest slot it has to keep),
// so the records a call forwarded are still in the ring afterwards and
// k_out_compact gathers the sent batch from there -- no staging copy.
enum : uint32_t { E_ORDER = 128 };

struct OutboundArgs {
  const uint32_t* host_off;
  uint32_t H, E;
  const uint64_t* time;
  const uint32_t *pkt, *len, *payload, *dst;
  const uint32_t* host_ip;
  uint32_t *head, *tail;
  uint4* ring;  // {packet, len, dst, payload_len}
  uint32_t cap;
  uint8_t* rflags;
  uint64_t* task_time;
  uint64_t *tb_cap, *tb_bal, *tb_inc, *tb_last;
  uint64_t window_end, bootstrap_end, sim_end;
  uint64_t* event_ctr;
  uint64_t* fwd_time;
  uint8_t* status;
  uint32_t n_status;
  uint32_t* start;  // per host: the first ring slot this call forwarded from
  const uint64_t *ev_id, *ev_born;  // per send (KEYED): the sending event's id and creation time
  uint64_t *task_id, *task_born;    // per host: the pending task's event id and creation time
  unsigned long long* blk;
  unsigned long long* bdiag = nullptr;  // as CodelArgs::bdiag
};

struct OutQ {
  uint32_t head, tail, oldest, mask, ip;
  uint4* ring;
  uint4 hr;  // the head record (valid while head < tail), loaded ahead of its pop
  uint4 cr;  // the relay's cached record (valid while R_CACHED): the slot at head - 1
  uint32_t sent;
  uint32_t err;
  // Staged window: the records pushed since begin_window() are the chunk's
  // send records wb, wb + 1, ... in LDS, so a head pushed there is read from
  // LDS instead of being re-read from the ring this lane just wrote (a forward
  // task pops back to back: each HBM re-read was a full round trip on the chain).
  bool win;
  uint32_t t0, wb;
  const __attribute__((address_space(3))) uint4* wr;
  __device__ void begin_window(const __attribute__((address_space(3))) uint4* r, uint32_t first) {
    win = true;
    t0 = tail;
    wb = first;
    wr = r;
  }
  __device__ void load_head() {
    if (head == tail) return;
    const uint32_t j = head - t0;
    if (win && j < tail - t0) {
      const __attribute__((address_space(3))) uint32_t* w =
          (const __attribute__((address_space(3))) uint32_t*)(wr + wb + j);
      hr = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      hr = ring[head & mask];
    }
  }
};

// The relay's forward task at `now` (run_forward_task -> forward_until_blocked),
// the interface as its source.
__device__ void out_task(OutQ& q, Relay& r, uint64_t now, const OutboundArgs& a, uint64_t& ctr_inc) {
  r.rf &= (uint8_t)~R_PENDING;
  for (;;) {
    uint4 rec;
    if (r.rf & R_CACHED) {  // next_packet.take(): the slot at head - 1
      rec = q.cr;
      r.rf &= (uint8_t)~R_CACHED;
    } else {
      if (q.head == q.tail) return;  // the interface has nothing: Idle
      rec = q.hr;
      q.head++;
      q.load_head();
    }
    const bool local = rec.z == q.ip;
    uint64_t wait;
    if (!local && now >= a.bootstrap_end && !r.remove(rec.y, now, wait)) {
      r.rf |= R_CACHED;  // RelayCached; forward_later(wait)
      q.cr = rec;
      r.schedule(now, now > ~0ull - wait ? ~0ull : now + wait, a.sim_end, ctr_inc);
      return;
    }
    if (rec.x < a.n_status) {
      a.status[rec.x] = local ? SG_OUT_LOCAL : SG_OUT_SENT;
      a.fwd_time[rec.x] = now;
    } else {
      q.err |= E_PKT;
    }
    q.sent += local ? 0 : 1;
  }
}

// KEYED: the sends carry their event's (creation time, id), and a task due at
// a send's own time runs first iff it was created before the sending event
// (Local events run in id = creation order, event.rs:163-183; a Packet event's
// send, id UINT64_MAX, precedes every Local event, event.rs:103-112).  Without
// keys every send precedes a task at its time.  A Local send's id also moves
// the host counter past it, so the tasks it schedules are numbered after it.  The keys cost 16 B of LDS per
// staged send, so the keyed chunk is smaller (40 B per send, 20 KB).
template <bool KEYED, int LM>
__global__ void __launch_bounds__(CD_THREADS) k_outbound(OutboundArgs a) {
  constexpr bool ANY = LM != 0;
  constexpr uint32_t CH = KEYED ? 512 : CD_OUT_CHUNK;
  const uint64_t d_t0 = a.bdiag ? wall_clock64() : 0;
  uint64_t d_walk = 0;
  __shared__ uint64_t s_t[CH];
  __shared__ uint4 s_r[CH];
  __shared__ uint64_t s_id[KEYED ? CH : 1], s_born[KEYED ? CH : 1];
  const uint32_t h0 = blockIdx.x * CD_HOSTS, t = threadIdx.x;
  const uint32_t h = h0 + t;
  const bool walker = t < CD_HOSTS && h < a.H;
  uint32_t hb = 0, he = 0;
  OutQ q{};
  Relay r{};
  uint64_t ctr_inc = 0, last = 0, last_born = 0, last_id = 0;
  if (walker) {
    hb = min(a.host_off[h], a.E);
    he = max(min(a.host_off[h + 1], a.E), hb);
    q.head = a.head[h];
    q.tail = a.tail[h];
    q.mask = a.cap - 1;
    q.ip = a.host_ip[h];
    q.ring = a.ring + (size_t)h * a.cap;
    r.rf = a.rflags[h];
    r.tt = a.task_time[h];
    r.cap = a.tb_cap[h];
    r.bal = a.tb_bal[h];
    r.set_inc(a.tb_inc[h]);
    r.last = a.tb_last[h];
    r.ctr0 = a.event_ctr ? a.event_ctr[h] : 0;
    r.tid = a.task_id[h];
    r.tborn = a.task_born[h];
    q.oldest = q.head - ((r.rf & R_CACHED) ? 1u : 0u);
    if (r.rf & R_CACHED) q.cr = q.ring[(q.head - 1) & q.mask];
    q.load_head();
  }
  // the block's events [p0, p1): lane 0's first and the last host's end, read from the
  // walkers' registers (loads of their own were waited for ahead of the walkers' state
  // loads once the chunk loop used them as scalars: a round trip per block, C4 +2.4 us)
  const uint32_t p0 = (uint32_t)__builtin_amdgcn_readlane((int)hb, 0);
  const uint32_t p1 = (uint32_t)__builtin_amdgcn_readlane((int)he, (int)min(CD_HOSTS - 1u, a.H - 1u - h0));
  auto due = [&](uint64_t before) { return (r.rf & R_PENDING) && !(r.rf & R_NEVER) && r.tt < before; };
  // a task at the send's own time that runs first: created before the sending Local event
  auto due_tie = [&](uint64_t now, uint64_t born, uint64_t id) {
    return KEYED && (r.rf & R_PENDING) && !(r.rf & R_NEVER) && r.tt == now && id != ~0ull &&
           (r.tborn < born || (r.tborn == born && r.tid < id));
  };
  if constexpr (!ANY) {  // contiguous chunks only: the r04 loop as it was (see with_chunk_map)
  for (uint32_t c0 = p0; c0 < p1; c0 += CH) {
    const uint32_t c1 = min(c0 + CH, p1);
    {
      uint64_t rt[CD_UNROLL], ri[KEYED ? CD_UNROLL : 1], rb[KEYED ? CD_UNROLL : 1];
      uint4 rr[CD_UNROLL];
      stage_chunk(
          c0, c1,
          [&](uint32_t i, int u) {
            rt[u] = a.time[i];
            rr[u] = make_uint4(a.pkt[i], a.len[i], a.dst[i], a.payload[i]);
            if constexpr (KEYED) {
              ri[u] = a.ev_id[i];
              rb[u] = a.ev_born[i];
            }
          },
          [&](uint32_t k, int u) {
            s_t[k] = rt[u];
            s_r[k] = rr[u];
            if constexpr (KEYED) {
              s_id[k] = ri[u];
              s_born[k] = rb[u];
            }
          });
    }
    __syncthreads();
    if (walker) {
      const uint32_t b = max(hb, c0), e = min(he, c1);
      const uint64_t d_w0 = a.bdiag ? clock64() : 0;
      q.begin_window((const __attribute__((address_space(3))) uint4*)s_r, b - c0);
      for (uint32_t i = b; i < e; i++) {
        const uint32_t k = i - c0;
        const uint64_t now = s_t[k];
        if (now >= a.window_end) q.err |= E_WINDOW;
        if (now < last) q.err |= E_ORDER;
        if constexpr (KEYED) {
          // execution order within a time: Packet-event sends, then Local ones by (created, id)
          const uint64_t id = s_id[k], born = s_born[k];
          if (now == last && i > hb) {
            const bool pk = id == ~0ull, lpk = last_id == ~0ull;
            if ((pk && !lpk) || (!pk && !lpk && (born < last_born || (born == last_born && id < last_id))))
              q.err |= E_ORDER;
          }
          last_born = born;
          last_id = id;
          // The sending event exists from its creation on, so the host's counter is past its id
          // (a Lamport-clock step; a no-op when the caller's ids come from this counter): before
          // a task that runs after that creation time (it may reschedule itself; at the time itself
          // the order of the task and the creating event is unknown), and
          // before the send (a task the send schedules takes a later id)
          while (due(now) || due_tie(now, born, id)) {
            if (id != ~0ull && r.tt > born && id - r.ctr0 >= ctr_inc && id >= r.ctr0) ctr_inc = id + 1 - r.ctr0;
            out_task(q, r, r.tt, a, ctr_inc);
          }
          // a send whose key equals the pending task's is no event order (two events, one id)
          if (id != ~0ull && (r.rf & R_PENDING) && !(r.rf & R_NEVER) && r.tt == now && r.tborn == born && r.tid == id)
            q.err |= E_ORDER;
          if (id != ~0ull && id - r.ctr0 >= ctr_inc && id >= r.ctr0) ctr_inc = id + 1 - r.ctr0;
        } else {
          while (due(now)) out_task(q, r, r.tt, a, ctr_inc);
        }
        last = now;
        if (q.tail - q.oldest >= a.cap) {  // the push would overwrite a slot this call still needs
          q.err |= E_FULL;
          continue;
        }
        // NetworkInterface::add_data_source: the record is the window's next element (read
        // from LDS at the head); the ring receives the window's records at the chunk's end
        // (k_out_compact gathers the sent ones from there) -- a ring store per send made the
        // walk's next vector-memory wait include it
        if (q.head == q.tail) q.hr = s_r[k];
        q.tail++;
        if (!(r.rf & R_PENDING)) r.schedule(now, now, a.sim_end, ctr_inc);  // notify: Idle -> forward_later(ZERO)
      }
      for (uint32_t j = 0; j < q.tail - q.t0; j++) q.ring[(q.t0 + j) & q.mask] = s_r[q.wb + j];
      if (a.bdiag) d_walk += clock64() - d_w0;
      q.win = false;  // the next chunk's staging overwrites the window
    }
    __syncthreads();
  }
  } else {
  __shared__ uint32_t s_hb[CD_HOSTS], s_hn[CD_HOSTS];
  uint32_t h_act;
  const uint32_t max_n = lane_major_setup<ANY>(hb, he - hb, s_hb, s_hn, h_act);
  with_chunk_map<ANY, CH>(ANY && lane_major_block<CH>(LM, p1 - p0, max_n, h_act), p0, p1, s_hb, s_hn,
                          [&](auto cm) {
  for (uint32_t c = 0; cm.has(c, max_n); c++) {
    const uint32_t clen = cm.len(c);
    for (uint32_t base = 0; base < clen; base += CD_THREADS * CD_UNROLL) {  // staging (see ChunkMap)
      uint64_t rt[CD_UNROLL], ri[KEYED ? CD_UNROLL : 1], rb[KEYED ? CD_UNROLL : 1];
      uint4 rr[CD_UNROLL];
      bool ok[CD_UNROLL];
#pragma unroll
      for (int u = 0; u < CD_UNROLL; u++) {
        const uint32_t i = cm.event(c, base + u * CD_THREADS + t, ok[u]);
        rt[u] = a.time[i];
        rr[u] = make_uint4(a.pkt[i], a.len[i], a.dst[i], a.payload[i]);
        if constexpr (KEYED) {
          ri[u] = a.ev_id[i];
          rb[u] = a.ev_born[i];
        }
      }
#pragma unroll
      for (int u = 0; u < CD_UNROLL; u++) {
        const uint32_t k = base + u * CD_THREADS + t;
        if (k < clen && ok[u]) {
          s_t[k] = rt[u];
          s_r[k] = rr[u];
          if constexpr (KEYED) {
            s_id[k] = ri[u];
            s_born[k] = rb[u];
          }
        }
      }
    }
    __syncthreads();
    if (walker) {
      uint32_t kb, ke, ib;
      cm.host_range(c, t, hb, he, kb, ke, ib);
      const uint64_t d_w0 = a.bdiag ? clock64() : 0;
      q.begin_window((const __attribute__((address_space(3))) uint4*)s_r, kb);
      for (uint32_t k = kb; k < ke; k++) {
        const uint32_t i = ib + (k - kb);
        const uint64_t now = s_t[k];
        if (now >= a.window_end) q.err |= E_WINDOW;
        if (now < last) q.err |= E_ORDER;
        if constexpr (KEYED) {
          // execution order within a time: Packet-event sends, then Local ones by (created, id)
          const uint64_t id = s_id[k], born = s_born[k];
          if (now == last && i > hb) {
            const bool pk = id == ~0ull, lpk = last_id == ~0ull;
            if ((pk && !lpk) || (!pk && !lpk && (born < last_born || (born == last_born && id < last_id))))
              q.err |= E_ORDER;
          }
          last_born = born;
          last_id = id;
          // The sending event exists from its creation on, so the host's counter is past its id
          // (a Lamport-clock step; a no-op when the caller's ids come from this counter): before
          // a task that runs after that creation time (it may reschedule itself; at the time itself
          // the order of the task and the creating event is unknown), and
          // before the send (a task the send schedules takes a later id)
          while (due(now) || due_tie(now, born, id)) {
            if (id != ~0ull && r.tt > born && id - r.ctr0 >= ctr_inc && id >= r.ctr0) ctr_inc = id + 1 - r.ctr0;
            out_task(q, r, r.tt, a, ctr_inc);
          }
          // a send whose key equals the pending task's is no event order (two events, one id)
          if (id != ~0ull && (r.rf & R_PENDING) && !(r.rf & R_NEVER) && r.tt == now && r.tborn == born && r.tid == id)
            q.err |= E_ORDER;
          if (id != ~0ull && id - r.ctr0 >= ctr_inc && id >= r.ctr0) ctr_inc = id + 1 - r.ctr0;
        } else {
          while (due(now)) out_task(q, r, r.tt, a, ctr_inc);
        }
        last = now;
        if (q.tail - q.oldest >= a.cap) {  // the push would overwrite a slot this call still needs
          q.err |= E_FULL;
          continue;
        }
        // NetworkInterface::add_data_source: the record is the window's next element (read
        // from LDS at the head); the ring receives the window's records at the chunk's end
        // (k_out_compact gathers the sent ones from there) -- a ring store per send made the
        // walk's next vector-memory wait include it
        if (q.head == q.tail) q.hr = s_r[k];
        q.tail++;
        if (!(r.rf & R_PENDING)) r.schedule(now, now, a.sim_end, ctr_inc);  // notify: Idle -> forward_later(ZERO)
      }
      for (uint32_t j = 0; j < q.tail - q.t0; j++) q.ring[(q.t0 + j) & q.mask] = s_r[q.wb + j];
      if (a.bdiag) d_walk += clock64() - d_w0;
      q.win = false;  // the next chunk's staging overwrites the window
    }
    __syncthreads();
  }
  });
  }
  unsigned long long err = 0, sent = 0;
  if (walker) {
    while (due(a.window_end)) out_task(q, r, r.tt, a, ctr_inc);
    a.head[h] = q.head;
    a.tail[h] = q.tail;
    a.rflags[h] = r.rf;
    a.task_time[h] = r.tt;
    a.tb_bal[h] = r.bal;
    a.tb_last[h] = r.last;
    a.task_id[h] = r.tid;
    a.task_born[h] = r.tborn;
    a.start[h] = q.oldest;
    if (a.event_ctr && ctr_inc) a.event_ctr[h] += ctr_inc;
    err = q.err;
    sent = q.sent;
  }
  lane_diag_store(a.bdiag, d_t0, d_walk, he - hb);
  if (t < 64) {
    for (int d = 32; d > 0; d >>= 1) {
      sent += __shfl_xor(sent, d, 64);
      err |= __shfl_xor(err, d, 64);
    }
    if (t == 0) {
      a.blk[2 * blockIdx.x] = sent;
      a.blk[2 * blockIdx.x + 1] = err;
    }
  }
}

// Exclusive prefix of the k_outbound blocks' sent counts (blk[2b]) -> boff[b]:
// where each block's slice of the sent batch starts; and k_codel_reduce's sums
// (the total sent, the error flags) into the mapped return block, in the same
// launch.  One block.
__global__ void __launch_bounds__(1024) k_blk_offsets(const unsigned long long* __restrict__ blk, uint32_t nb,
                                                      uint32_t* __restrict__ boff,
                                                      const uint32_t* __restrict__ group_err,
                                                      unsigned long long* __restrict__ ret) {
  __shared__ uint32_t wsum[16];
  __shared__ unsigned long long esum[16];
  __shared__ uint32_t carry;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t == 0) carry = 0;
  __syncthreads();
  unsigned long long e = 0;
  for (uint32_t c0 = 0; c0 < nb; c0 += 1024) {
    const uint32_t i = c0 + t;
    const uint32_t v = i < nb ? (uint32_t)blk[2 * i] : 0;
    if (i < nb) e |= blk[2 * i + 1];
    uint32_t x = v;  // inclusive wave scan
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t before = carry;
    for (uint32_t w = 0; w < wv; w++) before += wsum[w];
    if (i < nb) boff[i] = before + x - v;
    __syncthreads();
    if (t == 1023) carry = before + x;
    __syncthreads();
  }
  for (int s = 32; s > 0; s >>= 1) e |= __shfl_xor(e, s, 64);
  if (lane == 0) esum[wv] = e;
  __syncthreads();
  if (t == 0) {
    for (int w = 1; w < 16; w++) e |= esum[w];
    ret[0] = carry;  // the sent total (k_codel_reduce's sum)
    ret[1] = e | *group_err;
  }
}

// The sent batch: block b owns hosts [64b, 64b + 64), whose forwarded records
// are ring slots [start, end) per host (end = head, less a packet cached at the
// end).  The block walks the hosts' slot ranges as one concatenated sequence,
// 256 slots per step (coalesced within a host's range), skips local packets
// (a ballot prefix gives each kept record its rank) and writes its slice
// [boff[b], boff[b] + sent) of the batch with coalesced stores.
__global__ void __launch_bounds__(256) k_out_compact(uint32_t H, const uint32_t* __restrict__ start,
                                                     const uint32_t* __restrict__ head,
                                                     const uint8_t* __restrict__ rflags,
                                                     const uint32_t* __restrict__ host_ip,
                                                     const uint4* __restrict__ ring, uint32_t cap,
                                                     const uint64_t* __restrict__ fwd_time, uint32_t n_status,
                                                     const uint32_t* __restrict__ boff, sg_outbound_sent out) {
  __shared__ uint32_t s_off[CD_HOSTS + 1], s_start[CD_HOSTS], s_ip[CD_HOSTS];
  __shared__ uint32_t wsum[4];
  const uint32_t h0 = blockIdx.x * CD_HOSTS, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t < 64) {  // one wave: per-host slot counts and their exclusive prefix
    const uint32_t h = h0 + t;
    uint32_t len = 0;
    if (h < H) {
      const uint32_t st = start[h], end = head[h] - ((rflags[h] & R_CACHED) ? 1u : 0u);
      len = end - st;
      s_start[t] = st;
      s_ip[t] = host_ip[h];
    }
    uint32_t x = len;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= (uint32_t)d) x += y;
    }
    s_off[t + 1] = x;
    if (t == 0) s_off[0] = 0;
  }
  __syncthreads();
  const uint32_t S = s_off[CD_HOSTS], mask = cap - 1;
  uint32_t o = boff[blockIdx.x];
  // CU rounds of 256 records per step: every round's ring and forward-time loads are
  // issued (branch-free, clamped to a valid record) before the step's first store --
  // a load after a store waited for the store too
  constexpr int CU = 4;
  for (uint32_t j0 = 0; j0 < S; j0 += 256 * CU) {
    uint4 rec[CU];
    uint32_t kk[CU];
    bool keep[CU];
    uint64_t ft[CU];
#pragma unroll
    for (int u = 0; u < CU; u++) {
      const uint32_t j = j0 + u * 256 + t, jc = min(j, S - 1);
      uint32_t lo = 0, hi = CD_HOSTS;  // the host k with s_off[k] <= jc < s_off[k + 1]
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_off[mid] <= jc) lo = mid;
        else hi = mid;
      }
      kk[u] = lo;
      rec[u] = ring[(size_t)(h0 + lo) * cap + ((s_start[lo] + (jc - s_off[lo])) & mask)];
    }
#pragma unroll
    for (int u = 0; u < CU; u++) {
      keep[u] = j0 + u * 256 + t < S && rec[u].z != s_ip[kk[u]];
      ft[u] = n_status ? fwd_time[rec[u].x < n_status ? rec[u].x : 0u] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < CU; u++) {
      if (j0 + u * 256 >= S) break;
      const uint64_t m = __ballot(keep[u]);
      if (lane == 0) wsum[wv] = (uint32_t)__popcll(m);
      __syncthreads();
      uint32_t pos = o + (uint32_t)__popcll(m & ((1ull << lane) - 1));
      for (uint32_t w = 0; w < wv; w++) pos += wsum[w];
      if (keep[u] && pos < out.cap) {
        out.src_host[pos] = h0 + kk[u];
        out.dst_ipv4[pos] = rec[u].z;
        out.payload_len[pos] = rec[u].w;
        out.send_time_ns[pos] = rec[u].x < n_status ? ft[u] : 0;
        out.packet[pos] = rec[u].x;
      }
      o += wsum[0] + wsum[1] + wsum[2] + wsum[3];
      __syncthreads();
    }
  }
}

}  // namespace
}  // namespace sg

extern "C" {

int32_t sg_codel_create(sg_ctx* ctx, uint32_t n_hosts, uint32_t ring_cap, sg_codel** out) {
  if (!out) return SG_ERR_INVALID_ARG;
  *out = nullptr;
  sg_codel* q = nullptr;
  int32_t rc = sg::guarded(ctx, [&] {
    using namespace sg;
    if (ring_cap == 0 || ring_cap > (1u << 30)) throw Error(SG_ERR_INVALID_ARG, "ring_cap must be in [1, 2^30]");
    uint32_t cap = 1;
    while (cap < ring_cap) cap <<= 1;
    q = new sg_codel();
    q->ctx = ctx;
    q->n = n_hosts;
    q->cap = cap;
    const size_t n = std::max<uint32_t>(n_hosts, 1), r = n * cap;
    SG_HIP(hipMalloc(&q->flags, n));
    SG_HIP(hipMalloc(&q->iend, n * 8));
    SG_HIP(hipMalloc(&q->dnext, n * 8));
    SG_HIP(hipMalloc(&q->cur, n * 8));
    SG_HIP(hipMalloc(&q->prev, n * 8));
    SG_HIP(hipMalloc(&q->bytes, n * 8));
    SG_HIP(hipMalloc(&q->head, n * 4));
    SG_HIP(hipMalloc(&q->tail, n * 4));
    SG_HIP(hipMalloc(&q->ring, r * 16));
    SG_HIP(hipHostMalloc(&q->ret, 16, hipHostMallocMapped | hipHostMallocCoherent));
    hipStream_t st = ctx->stream;  // CoDelQueue::new (codel_queue.rs:85-95): empty, Store mode, no times
    SG_HIP(hipMemsetAsync(q->flags, 0, n, st));
    void* z8[] = {q->iend, q->dnext, q->cur, q->prev, q->bytes};
    for (void* p : z8) SG_HIP(hipMemsetAsync(p, 0, n * 8, st));
    SG_HIP(hipMemsetAsync(q->head, 0, n * 4, st));
    SG_HIP(hipMemsetAsync(q->tail, 0, n * 4, st));
    SG_HIP(hipStreamSynchronize(st));
  });
  if (rc != SG_OK) {
    delete q;
    return rc;
  }
  *out = q;
  return SG_OK;
}

void sg_codel_destroy(sg_codel* q) {
  if (!q) return;
  if (q->ctx) (void)hipSetDevice(q->ctx->device);
  delete q;
}

uint32_t sg_codel_ring_cap(const sg_codel* q) { return q ? q->cap : 0; }

}  // extern "C"

struct sg_inbound {
  sg_codel* q = nullptr;
  uint8_t* rflags = nullptr;
  uint64_t* task_time = nullptr;
  uint64_t *task_id = nullptr, *task_born = nullptr;
  uint32_t *cached_pkt = nullptr, *cached_len = nullptr;
  uint64_t *tb_cap = nullptr, *tb_bal = nullptr, *tb_inc = nullptr, *tb_last = nullptr;
  ~sg_inbound() {
    void* ps[] = {rflags, task_time, task_id, task_born, cached_pkt, cached_len, tb_cap, tb_bal, tb_inc, tb_last};
    for (void* p : ps)
      if (p) (void)hipFree(p);
    sg_codel_destroy(q);
  }
};

// SG_LANE_MAJOR: the chunk layout of the lane kernels (ChunkMap): 0 contiguous, 1 lane-major,
// unset / 2 by each block's event count (tests force both on the same events)
int lane_major_env() {
  const char* e = getenv("SG_LANE_MAJOR");
  return e && *e ? std::max(0, std::min(2, atoi(e))) : 2;
}

// The lane-major layout is compiled into a launch when forced (SG_LANE_MAJOR=1) or when
// the blocks average more than two contiguous chunks of ch events (C5: ~12.8k codel events
// per block; C4: ~1.3k, which keeps the contiguous-only kernel)
int lane_major_launch(int mode, size_t n_events, uint32_t nb, uint32_t ch) {
  return mode == 1 ? 1 : (mode == 2 && n_events > 2ull * ch * nb) ? 2 : 0;
}

// SG_LANE_DIAG=1: per-block timing of the lane-per-host kernels on stderr (a
// diagnostic: a synchronous copy after the launch; never set in a measured run)
unsigned long long* lane_diag_alloc(uint32_t nb) {
  const char* e = getenv("SG_LANE_DIAG");
  if (!e || atoi(e) == 0) return nullptr;
  unsigned long long* d = nullptr;
  SG_HIP(hipMalloc(&d, (size_t)nb * 32));
  SG_HIP(hipMemset(d, 0, (size_t)nb * 32));
  return d;
}
void lane_diag_report(hipStream_t st, const char* name, unsigned long long* d, uint32_t nb) {
  if (!d) return;
  std::vector<unsigned long long> h((size_t)nb * 4);
  SG_HIP(hipStreamSynchronize(st));
  SG_HIP(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
  (void)hipFree(d);
  uint64_t t_min = ~0ull, t_max = 0, s_max = 0;
  std::vector<double> dur(nb), walk(nb), ev(nb);
  for (uint32_t b = 0; b < nb; b++) {
    t_min = std::min<uint64_t>(t_min, h[4 * b]);
    t_max = std::max<uint64_t>(t_max, h[4 * b + 1]);
  }
  for (uint32_t b = 0; b < nb; b++) {
    s_max = std::max<uint64_t>(s_max, h[4 * b] - t_min);
    dur[b] = (h[4 * b + 1] - h[4 * b]) * 0.01;  // 100 MHz -> us
    walk[b] = h[4 * b + 2] / 2400.0;              // shader clock cycles -> us at ~2.4 GHz
    ev[b] = (double)h[4 * b + 3];
  }
  auto q = [](std::vector<double> v, double f) {
    std::sort(v.begin(), v.end());
    return v[(size_t)std::min<double>(v.size() - 1, f * v.size())];
  };
  double mw = 0, me = 0;
  for (uint32_t b = 0; b < nb; b++) mw += walk[b] / nb, me += ev[b] / nb;
  uint32_t slow = 0;  // the slowest block (its hosts are [64 slow, 64 slow + 64))
  for (uint32_t b = 1; b < nb; b++)
    if (dur[b] > dur[slow]) slow = b;
  fprintf(stderr,
          "[lane] %s: %u blocks, span %.2f us, last start +%.2f us; block us p50 %.2f p90 %.2f max %.2f; "
          "walk us (busiest lane) mean %.2f max %.2f; busiest-lane events mean %.1f max %.0f; slowest block %u "
          "(walk %.2f us, busiest lane %.0f events)\n",
          name, nb, (t_max - t_min) * 0.01, s_max * 0.01, q(dur, 0.5), q(dur, 0.9), q(dur, 1.0), mw, q(walk, 1.0), me,
          q(ev, 1.0), slow, walk[slow], ev[slow]);
}

extern "C" {

int32_t sg_codel_run(sg_ctx* ctx, sg_codel* q, const sg_codel_events* ev, uint32_t* pop_result,
                     uint8_t* pkt_status, uint32_t n_packets, uint64_t* n_dropped) {
  return sg::guarded(ctx, [&] {
    using namespace sg;
    if (!q || q->ctx != ctx || !ev) throw Error(SG_ERR_INVALID_ARG, "null argument");
    const uint32_t E = ev->n_events, H = q->n;
    if (n_dropped) *n_dropped = 0;
    if (!E) return;
    if (!ev->host || !ev->kind || !ev->time_ns || !ev->packet || !ev->len || !pop_result ||
        (n_packets && !pkt_status))
      throw Error(SG_ERR_INVALID_ARG, "null event or output array");
    hipStream_t st = ctx->stream;
    uint32_t* ws = ctx->d_seg.get<uint32_t>((size_t)H + 8);  // [offsets H+1][grouping error]
    uint32_t* gerr = ws + (size_t)H + 1;
    SG_HIP(hipMemsetAsync(gerr, 0, 4, st));
    launch_group_offsets(ctx, ev->host, E, H, ws, gerr);
    const uint32_t nb = std::max<uint32_t>(1, (H + CD_HOSTS - 1) / CD_HOSTS);
    CodelArgs a{ws, H, E, ev->kind, ev->time_ns, ev->packet, ev->len, q->flags, q->iend, q->dnext, q->cur,
                q->prev, q->bytes, q->head, q->tail, q->ring, q->cap, pop_result,
                pkt_status, n_packets, ctx->d_blk.get<unsigned long long>(2 * (size_t)nb)};
    a.bdiag = lane_diag_alloc(nb);
    {
      // per event: 17 B in, 4 B result, ring slot 16 B written (push) or read (pop), 1 B status
      TimedLaunch tl(ctx, "codel", 38.0 * E + 56.0 * H);
      const int lm = lane_major_launch(lane_major_env(), E, nb, CD_CHUNK);
      if (lm == 2)
        hipLaunchKernelGGL(k_codel<2>, dim3(nb), dim3(CD_THREADS), 0, st, a);
      else if (lm == 1)
        hipLaunchKernelGGL(k_codel<1>, dim3(nb), dim3(CD_THREADS), 0, st, a);
      else
        hipLaunchKernelGGL(k_codel<0>, dim3(nb), dim3(CD_THREADS), 0, st, a);
    }
    lane_diag_report(st, "k_codel", a.bdiag, nb);
    hipLaunchKernelGGL(k_codel_reduce, dim3(1), dim3(1024), 0, st, a.blk, nb, gerr, q->ret);
    SG_CHECK_LAUNCH();
    SG_HIP(hipStreamSynchronize(st));
    const volatile unsigned long long* r = q->ret;
    const uint64_t err = r[1];
    if (err & E_UNSORTED) throw Error(SG_ERR_UNSORTED, "CoDel events must be grouped by ascending host");
    if (err & E_HOST) throw Error(SG_ERR_INVALID_ARG, "CoDel event host out of range");
    if (err & E_FULL) throw Error(SG_ERR_CAPACITY, "a CoDel queue outgrew its ring (raise ring_cap)");
    if (err & E_PKT) throw Error(SG_ERR_INVALID_ARG, "CoDel packet id >= n_packets");
    if (n_dropped) *n_dropped = r[0];
  });
}

int32_t sg_codel_get_state(sg_codel* q, sg_codel_state* o) {
  if (!q || !o) return SG_ERR_INVALID_ARG;
  return sg::guarded(q->ctx, [&] {
    const size_t n = q->n, r = n * q->cap;
    hipStream_t st = q->ctx->stream;
    struct { void* h; const void* d; size_t b; } cp[] = {
        {o->flags, q->flags, n}, {o->interval_end, q->iend, n * 8}, {o->drop_next, q->dnext, n * 8},
        {o->cur_drops, q->cur, n * 8}, {o->prev_drops, q->prev, n * 8}, {o->bytes, q->bytes, n * 8},
        {o->head, q->head, n * 4}, {o->tail, q->tail, n * 4}};
    for (auto& c : cp)
      if (c.h && c.b) SG_HIP(hipMemcpyAsync(c.h, c.d, c.b, hipMemcpyDeviceToHost, st));
    std::vector<uint4> ring(r);
    if (r) SG_HIP(hipMemcpyAsync(ring.data(), q->ring, r * 16, hipMemcpyDeviceToHost, st));
    SG_HIP(hipStreamSynchronize(st));
    for (size_t i = 0; i < r; i++) {
      if (o->ring_packet) o->ring_packet[i] = ring[i].x;
      if (o->ring_len) o->ring_len[i] = ring[i].y;
      if (o->ring_time) o->ring_time[i] = ((uint64_t)ring[i].w << 32) | ring[i].z;
    }
  });
}

int32_t sg_codel_set_state(sg_codel* q, const sg_codel_state* in) {
  if (!q || !in) return SG_ERR_INVALID_ARG;
  return sg::guarded(q->ctx, [&] {
    const size_t n = q->n, r = n * q->cap;
    hipStream_t st = q->ctx->stream;
    struct { void* d; const void* h; size_t b; } cp[] = {
        {q->flags, in->flags, n}, {q->iend, in->interval_end, n * 8}, {q->dnext, in->drop_next, n * 8},
        {q->cur, in->cur_drops, n * 8}, {q->prev, in->prev_drops, n * 8}, {q->bytes, in->bytes, n * 8},
        {q->head, in->head, n * 4}, {q->tail, in->tail, n * 4}};
    for (auto& c : cp)
      if (c.h && c.b) SG_HIP(hipMemcpyAsync(c.d, c.h, c.b, hipMemcpyHostToDevice, st));
    if (in->ring_packet && in->ring_time && in->ring_len && r) {
      std::vector<uint4> ring(r);
      for (size_t i = 0; i < r; i++)
        ring[i] = make_uint4(in->ring_packet[i], in->ring_len[i], (uint32_t)in->ring_time[i],
                             (uint32_t)(in->ring_time[i] >> 32));
      SG_HIP(hipMemcpyAsync(q->ring, ring.data(), r * 16, hipMemcpyHostToDevice, st));
      SG_HIP(hipStreamSynchronize(st));  // before `ring` goes out of scope
    }
    SG_HIP(hipStreamSynchronize(st));
  });
}

}  // extern "C"

extern "C" {

int32_t sg_inbound_create(sg_ctx* ctx, uint32_t n_hosts, const uint64_t* bw_down_bits, uint32_t ring_cap,
                          sg_inbound** out) {
  if (!out) return SG_ERR_INVALID_ARG;
  *out = nullptr;
  sg_inbound* ib = new (std::nothrow) sg_inbound();
  if (!ib) return SG_ERR_OOM;
  int32_t rc = sg_codel_create(ctx, n_hosts, ring_cap, &ib->q);
  if (rc == SG_OK)
    rc = sg::guarded(ctx, [&] {
      using namespace sg;
      if (n_hosts && !bw_down_bits) throw Error(SG_ERR_INVALID_ARG, "null bandwidth array");
      const size_t n = std::max<uint32_t>(n_hosts, 1);
      SG_HIP(hipMalloc(&ib->rflags, n));
      SG_HIP(hipMalloc(&ib->task_time, n * 8));
      SG_HIP(hipMalloc(&ib->task_id, n * 8));
      SG_HIP(hipMalloc(&ib->task_born, n * 8));
      SG_HIP(hipMalloc(&ib->cached_pkt, n * 4));
      SG_HIP(hipMalloc(&ib->cached_len, n * 4));
      SG_HIP(hipMalloc(&ib->tb_cap, n * 8));
      SG_HIP(hipMalloc(&ib->tb_bal, n * 8));
      SG_HIP(hipMalloc(&ib->tb_inc, n * 8));
      SG_HIP(hipMalloc(&ib->tb_last, n * 8));
      // Relay::new (relay/mod.rs:48-66): Idle, no cached packet, a full bucket
      std::vector<uint64_t> inc(n), cap(n), last(n, 946684800ull * 1000000000ull);  // EmulatedTime::SIMULATION_START
      for (uint32_t h = 0; h < n_hosts; h++) {
        inc[h] = std::max<uint64_t>(1, (bw_down_bits[h] / 8) / 1000);  // create_token_bucket (:296-304)
        cap[h] = inc[h] + CD_MTU;                                      // + get_burst_allowance (:306-309)
      }
      hipStream_t st = ctx->stream;
      SG_HIP(hipMemsetAsync(ib->rflags, 0, n, st));
      SG_HIP(hipMemsetAsync(ib->task_time, 0, n * 8, st));
      SG_HIP(hipMemsetAsync(ib->task_id, 0, n * 8, st));
      SG_HIP(hipMemsetAsync(ib->task_born, 0, n * 8, st));
      SG_HIP(hipMemsetAsync(ib->cached_pkt, 0, n * 4, st));
      SG_HIP(hipMemsetAsync(ib->cached_len, 0, n * 4, st));
      SG_HIP(hipMemcpyAsync(ib->tb_cap, cap.data(), n * 8, hipMemcpyHostToDevice, st));
      SG_HIP(hipMemcpyAsync(ib->tb_bal, cap.data(), n * 8, hipMemcpyHostToDevice, st));
      SG_HIP(hipMemcpyAsync(ib->tb_inc, inc.data(), n * 8, hipMemcpyHostToDevice, st));
      SG_HIP(hipMemcpyAsync(ib->tb_last, last.data(), n * 8, hipMemcpyHostToDevice, st));
      SG_HIP(hipStreamSynchronize(st));
    });
  if (rc != SG_OK) {
    delete ib;
    return rc;
  }
  *out = ib;
  return SG_OK;
}

void sg_inbound_destroy(sg_inbound* ib) {
  if (!ib) return;
  if (ib->q && ib->q->ctx) (void)hipSetDevice(ib->q->ctx->device);
  delete ib;
}

uint32_t sg_inbound_ring_cap(const sg_inbound* ib) { return ib ? ib->q->cap : 0; }

}  // extern "C"

namespace sg {
// sg_inbound_run / sg_inbound_run_ordered (arr_status set: outputs per arrival of this call)
static int32_t inbound_run(sg_ctx* ctx, sg_inbound* ib, const sg_inbound_arrivals* arr, uint64_t window_end_ns,
                           uint64_t bootstrap_end_ns, uint64_t sim_end_ns, uint64_t* event_ctr, uint64_t* fwd_time,
                           uint8_t* pkt_status, uint32_t n_packets, uint8_t* arr_status, uint64_t* arr_fwd,
                           uint64_t* n_dropped) {
  return sg::guarded(ctx, [&] {
    if (!ib || !arr || ib->q->ctx != ctx) throw Error(SG_ERR_INVALID_ARG, "null argument");
    sg_codel* q = ib->q;
    const uint32_t E = arr->n, H = q->n;
    const bool ord = arr_status != nullptr;
    if (n_dropped) *n_dropped = 0;
    if (E && (!arr->host || !arr->time_ns || !arr->packet || !arr->len))
      throw Error(SG_ERR_INVALID_ARG, "null arrival array");
    if (n_packets && (!pkt_status || !fwd_time)) throw Error(SG_ERR_INVALID_ARG, "null output array");
    if (ord && E && !arr_fwd) throw Error(SG_ERR_INVALID_ARG, "null arrival output array");
    if (ord && E >= ARR_BIT) throw Error(SG_ERR_INVALID_ARG, "too many arrivals for one ordered call");
    // packet ids stay below 2^31 (an ordered call tells its arrival indices by bit 31)
    if (n_packets > ARR_BIT) throw Error(SG_ERR_INVALID_ARG, "n_packets above 2^31");
    if (!H) return;
    hipStream_t st = ctx->stream;
    uint32_t* ws = ctx->d_seg.get<uint32_t>((size_t)H + 8);
    uint32_t* gerr = ws + (size_t)H + 1;
    SG_HIP(hipMemsetAsync(gerr, 0, 4, st));
    if (E) {
      launch_group_offsets(ctx, arr->host, E, H, ws, gerr);
    } else {
      SG_HIP(hipMemsetAsync(ws, 0, ((size_t)H + 1) * 4, st));  // no arrivals: pending tasks only
    }
    const uint32_t nb = (H + CD_HOSTS - 1) / CD_HOSTS;
    InboundArgs a;
    a.q = CodelArgs{ws, H, E, nullptr, arr->time_ns, arr->packet, arr->len, q->flags, q->iend, q->dnext, q->cur,
                    q->prev, q->bytes, q->head, q->tail, q->ring, q->cap, nullptr, pkt_status, n_packets,
                    ctx->d_blk.get<unsigned long long>(2 * (size_t)nb)};
    a.rflags = ib->rflags;
    a.task_time = ib->task_time;
    a.task_id = ib->task_id;
    a.task_born = ib->task_born;
    a.cached_pkt = ib->cached_pkt;
    a.cached_len = ib->cached_len;
    a.tb_cap = ib->tb_cap;
    a.tb_bal = ib->tb_bal;
    a.tb_inc = ib->tb_inc;
    a.tb_last = ib->tb_last;
    a.window_end = window_end_ns;
    a.bootstrap_end = bootstrap_end_ns;
    a.sim_end = sim_end_ns;
    a.event_ctr = event_ctr;
    a.fwd_time = fwd_time;
    a.arr_status = arr_status;
    a.arr_fwd = arr_fwd;
    {
      // per arrival: 16 B in, a 16-B ring record written and read, 9 B out (ordered: 12 B in, the
      // packet id read only for an element still queued at the end); per host: ~160 B of state
      a.q.bdiag = lane_diag_alloc(nb);
      TimedLaunch tl(ctx, "inbound", (ord ? 53.0 : 57.0) * E + 160.0 * H);
      const int lm = lane_major_launch(lane_major_env(), E, nb, CD_CHUNK);
      auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(nb), dim3(CD_THREADS), 0, st, a); };
      if (ord) {
        if (lm == 2) go(k_inbound<2, true>);
        else if (lm == 1) go(k_inbound<1, true>);
        else go(k_inbound<0, true>);
      } else {
        if (lm == 2) go(k_inbound<2>);
        else if (lm == 1) go(k_inbound<1>);
        else go(k_inbound<0>);
      }
    }
    lane_diag_report(st, "k_inbound", a.q.bdiag, nb);
    hipLaunchKernelGGL(k_codel_reduce, dim3(1), dim3(1024), 0, st, a.q.blk, nb, gerr, q->ret);
    SG_CHECK_LAUNCH();
    SG_HIP(hipStreamSynchronize(st));
    const volatile unsigned long long* r = q->ret;
    const uint64_t err = r[1];
    if (err & E_UNSORTED) throw Error(SG_ERR_UNSORTED, "arrivals must be grouped by ascending host");
    if (err & E_HOST) throw Error(SG_ERR_INVALID_ARG, "arrival host out of range");
    if (err & E_FULL) throw Error(SG_ERR_CAPACITY, "a CoDel queue outgrew its ring (raise ring_cap)");
    if (err & E_PKT) throw Error(SG_ERR_INVALID_ARG, "packet id >= n_packets");
    if (err & E_WINDOW) throw Error(SG_ERR_INVALID_ARG, "an arrival is at or after window_end");
    if (n_dropped) *n_dropped = r[0];
  });
}
}  // namespace sg

extern "C" {

int32_t sg_inbound_run(sg_ctx* ctx, sg_inbound* ib, const sg_inbound_arrivals* arr, uint64_t window_end_ns,
                       uint64_t bootstrap_end_ns, uint64_t sim_end_ns, uint64_t* event_ctr, uint64_t* fwd_time,
                       uint8_t* pkt_status, uint32_t n_packets, uint64_t* n_dropped) {
  return sg::inbound_run(ctx, ib, arr, window_end_ns, bootstrap_end_ns, sim_end_ns, event_ctr, fwd_time, pkt_status,
                         n_packets, nullptr, nullptr, n_dropped);
}

int32_t sg_inbound_run_ordered(sg_ctx* ctx, sg_inbound* ib, const sg_inbound_arrivals* arr, uint64_t window_end_ns,
                               uint64_t bootstrap_end_ns, uint64_t sim_end_ns, uint64_t* event_ctr,
                               uint64_t* fwd_time, uint8_t* pkt_status, uint32_t n_packets, uint64_t* arr_fwd_time,
                               uint8_t* arr_status, uint64_t* n_dropped) {
  if (arr && arr->n && !arr_status) return SG_ERR_INVALID_ARG;
  // (no arrivals: nothing is written per arrival, and the two kernels agree)
  return sg::inbound_run(ctx, ib, arr, window_end_ns, bootstrap_end_ns, sim_end_ns, event_ctr, fwd_time, pkt_status,
                         n_packets, arr && arr->n ? arr_status : nullptr, arr_fwd_time, n_dropped);
}

int32_t sg_inbound_get_state(sg_inbound* ib, sg_codel_state* queue, sg_inbound_relay_state* o) {
  if (!ib) return SG_ERR_INVALID_ARG;
  if (queue) {
    const int32_t rc = sg_codel_get_state(ib->q, queue);
    if (rc != SG_OK) return rc;
  }
  if (!o) return SG_OK;
  return sg::guarded(ib->q->ctx, [&] {
    const size_t n = ib->q->n;
    hipStream_t st = ib->q->ctx->stream;
    struct { void* h; const void* d; size_t b; } cp[] = {
        {o->flags, ib->rflags, n}, {o->task_time, ib->task_time, n * 8}, {o->cached_packet, ib->cached_pkt, n * 4},
        {o->cached_len, ib->cached_len, n * 4}, {o->tb_capacity, ib->tb_cap, n * 8},
        {o->tb_balance, ib->tb_bal, n * 8}, {o->tb_increment, ib->tb_inc, n * 8},
        {o->tb_last_refill, ib->tb_last, n * 8}, {o->task_event_id, ib->task_id, n * 8},
        {o->task_created_ns, ib->task_born, n * 8}};
    for (auto& c : cp)
      if (c.h && c.b) SG_HIP(hipMemcpyAsync(c.h, c.d, c.b, hipMemcpyDeviceToHost, st));
    SG_HIP(hipStreamSynchronize(st));
  });
}

}  // extern "C"

struct sg_outbound {
  sg_ctx* ctx = nullptr;
  uint32_t n = 0, cap = 0;
  uint32_t *host_ip = nullptr, *head = nullptr, *tail = nullptr, *start = nullptr, *off = nullptr;
  uint4* ring = nullptr;
  uint8_t* rflags = nullptr;
  uint64_t *task_time = nullptr, *tb_cap = nullptr, *tb_bal = nullptr, *tb_inc = nullptr, *tb_last = nullptr;
  uint64_t *task_id = nullptr, *task_born = nullptr;
  unsigned long long* ret = nullptr;  // pinned host-mapped: [sent, error flags]
  ~sg_outbound() {
    void* ps[] = {host_ip, head, tail, start, off, ring, rflags, task_time, task_id, task_born,
                  tb_cap, tb_bal, tb_inc, tb_last};
    for (void* p : ps)
      if (p) (void)hipFree(p);
    if (ret) (void)hipHostFree(ret);
  }
};

extern "C" {

int32_t sg_outbound_create(sg_ctx* ctx, uint32_t n_hosts, const uint32_t* host_ipv4, const uint64_t* bw_up_bits,
                           uint32_t ring_cap, sg_outbound** out) {
  if (!out) return SG_ERR_INVALID_ARG;
  *out = nullptr;
  sg_outbound* ob = nullptr;
  int32_t rc = sg::guarded(ctx, [&] {
    using namespace sg;
    if (ring_cap == 0 || ring_cap > (1u << 30)) throw Error(SG_ERR_INVALID_ARG, "ring_cap must be in [1, 2^30]");
    if (n_hosts && (!host_ipv4 || !bw_up_bits)) throw Error(SG_ERR_INVALID_ARG, "null address or bandwidth array");
    uint32_t cap = 1;
    while (cap < ring_cap) cap <<= 1;
    ob = new sg_outbound();
    ob->ctx = ctx;
    ob->n = n_hosts;
    ob->cap = cap;
    const size_t n = std::max<uint32_t>(n_hosts, 1);
    SG_HIP(hipMalloc(&ob->host_ip, n * 4));
    SG_HIP(hipMalloc(&ob->head, n * 4));
    SG_HIP(hipMalloc(&ob->tail, n * 4));
    SG_HIP(hipMalloc(&ob->start, n * 4));
    SG_HIP(hipMalloc(&ob->off, ((n + CD_HOSTS - 1) / CD_HOSTS + 1) * 4));  // per k_outbound block
    SG_HIP(hipMalloc(&ob->ring, n * cap * 16));
    SG_HIP(hipMalloc(&ob->rflags, n));
    SG_HIP(hipMalloc(&ob->task_time, n * 8));
    SG_HIP(hipMalloc(&ob->task_id, n * 8));
    SG_HIP(hipMalloc(&ob->task_born, n * 8));
    SG_HIP(hipMalloc(&ob->tb_cap, n * 8));
    SG_HIP(hipMalloc(&ob->tb_bal, n * 8));
    SG_HIP(hipMalloc(&ob->tb_inc, n * 8));
    SG_HIP(hipMalloc(&ob->tb_last, n * 8));
    SG_HIP(hipHostMalloc(&ob->ret, 16, hipHostMallocMapped | hipHostMallocCoherent));
    // Relay::new (relay/mod.rs:91-109): Idle, nothing cached, a full bucket;
    // the interface's queue empty
    std::vector<uint64_t> inc(n), tcap(n), last(n, 946684800ull * 1000000000ull);  // EmulatedTime::SIMULATION_START
    for (uint32_t h = 0; h < n_hosts; h++) {
      inc[h] = std::max<uint64_t>(1, (bw_up_bits[h] / 8) / 1000);  // create_token_bucket (:278-315)
      tcap[h] = inc[h] + CD_MTU;                                   // + get_burst_allowance (:317-319)
    }
    hipStream_t st = ctx->stream;
    if (n_hosts) SG_HIP(hipMemcpyAsync(ob->host_ip, host_ipv4, (size_t)n_hosts * 4, hipMemcpyHostToDevice, st));
    SG_HIP(hipMemsetAsync(ob->head, 0, n * 4, st));
    SG_HIP(hipMemsetAsync(ob->tail, 0, n * 4, st));
    SG_HIP(hipMemsetAsync(ob->rflags, 0, n, st));
    SG_HIP(hipMemsetAsync(ob->task_time, 0, n * 8, st));
    SG_HIP(hipMemsetAsync(ob->task_id, 0, n * 8, st));
    SG_HIP(hipMemsetAsync(ob->task_born, 0, n * 8, st));
    SG_HIP(hipMemcpyAsync(ob->tb_cap, tcap.data(), n * 8, hipMemcpyHostToDevice, st));
    SG_HIP(hipMemcpyAsync(ob->tb_bal, tcap.data(), n * 8, hipMemcpyHostToDevice, st));
    SG_HIP(hipMemcpyAsync(ob->tb_inc, inc.data(), n * 8, hipMemcpyHostToDevice, st));
    SG_HIP(hipMemcpyAsync(ob->tb_last, last.data(), n * 8, hipMemcpyHostToDevice, st));
    SG_HIP(hipStreamSynchronize(st));
  });
  if (rc != SG_OK) {
    delete ob;
    return rc;
  }
  *out = ob;
  return SG_OK;
}

void sg_outbound_destroy(sg_outbound* ob) {
  if (!ob) return;
  if (ob->ctx) (void)hipSetDevice(ob->ctx->device);
  delete ob;
}

uint32_t sg_outbound_ring_cap(const sg_outbound* ob) { return ob ? ob->cap : 0; }

int32_t sg_outbound_run(sg_ctx* ctx, sg_outbound* ob, const sg_outbound_sends* s, uint64_t window_end_ns,
                        uint64_t bootstrap_end_ns, uint64_t sim_end_ns, uint64_t* event_ctr, uint64_t* fwd_time,
                        uint8_t* pkt_status, uint32_t n_packets, sg_outbound_sent* sent, uint32_t* n_sent) {
  return sg::guarded(ctx, [&] {
    using namespace sg;
    if (!ob || !s || ob->ctx != ctx) throw Error(SG_ERR_INVALID_ARG, "null argument");
    const uint32_t E = s->n, H = ob->n;
    if (n_sent) *n_sent = 0;
    if (E && (!s->host || !s->time_ns || !s->packet || !s->len || !s->payload_len || !s->dst_ipv4))
      throw Error(SG_ERR_INVALID_ARG, "null send array");
    if (n_packets && (!pkt_status || !fwd_time)) throw Error(SG_ERR_INVALID_ARG, "null output array");
    const bool keyed = s->event_id != nullptr;
    if (keyed != (s->event_created_ns != nullptr))
      throw Error(SG_ERR_INVALID_ARG, "event_id and event_created_ns are given together or not at all");
    if (keyed && !event_ctr) throw Error(SG_ERR_INVALID_ARG, "send event ids need the hosts' event counters");
    if (sent && sent->cap && (!sent->src_host || !sent->dst_ipv4 || !sent->payload_len || !sent->send_time_ns ||
                              !sent->packet))
      throw Error(SG_ERR_INVALID_ARG, "null sent-batch array");
    if (!H) return;
    hipStream_t st = ctx->stream;
    uint32_t* ws = ctx->d_seg.get<uint32_t>((size_t)H + 8);
    uint32_t* gerr = ws + (size_t)H + 1;
    SG_HIP(hipMemsetAsync(gerr, 0, 4, st));
    if (E) {
      launch_group_offsets(ctx, s->host, E, H, ws, gerr);
    } else {
      SG_HIP(hipMemsetAsync(ws, 0, ((size_t)H + 1) * 4, st));  // no sends: pending tasks only
    }
    const uint32_t nb = (H + CD_HOSTS - 1) / CD_HOSTS;
    OutboundArgs a;
    a.host_off = ws;
    a.H = H;
    a.E = E;
    a.time = s->time_ns;
    a.pkt = s->packet;
    a.len = s->len;
    a.payload = s->payload_len;
    a.dst = s->dst_ipv4;
    a.host_ip = ob->host_ip;
    a.head = ob->head;
    a.tail = ob->tail;
    a.ring = ob->ring;
    a.cap = ob->cap;
    a.rflags = ob->rflags;
    a.task_time = ob->task_time;
    a.task_id = ob->task_id;
    a.task_born = ob->task_born;
    a.ev_id = s->event_id;
    a.ev_born = s->event_created_ns;
    a.tb_cap = ob->tb_cap;
    a.tb_bal = ob->tb_bal;
    a.tb_inc = ob->tb_inc;
    a.tb_last = ob->tb_last;
    a.window_end = window_end_ns;
    a.bootstrap_end = bootstrap_end_ns;
    a.sim_end = sim_end_ns;
    a.event_ctr = event_ctr;
    a.fwd_time = fwd_time;
    a.status = pkt_status;
    a.n_status = n_packets;
    a.start = ob->start;
    a.blk = ctx->d_blk.get<unsigned long long>(2 * (size_t)nb);
    {
      // per send: 24 B in, a 16-B ring record written and read, 9 B out; per host: ~90 B of state
      a.bdiag = lane_diag_alloc(nb);
        TimedLaunch tl(ctx, "outbound", 65.0 * E + 90.0 * H);
      const int lm = lane_major_launch(lane_major_env(), E, nb, keyed ? 512u : (uint32_t)CD_OUT_CHUNK);
      auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(nb), dim3(CD_THREADS), 0, st, a); };
      if (keyed && E)
        lm == 2 ? go(k_outbound<true, 2>) : lm == 1 ? go(k_outbound<true, 1>) : go(k_outbound<true, 0>);
      else
        lm == 2 ? go(k_outbound<false, 2>) : lm == 1 ? go(k_outbound<false, 1>) : go(k_outbound<false, 0>);
    }
    lane_diag_report(st, "k_outbound", a.bdiag, nb);
    if (sent) {  // the blocks' offsets and the sums in one launch, then the compaction
      hipLaunchKernelGGL(k_blk_offsets, dim3(1), dim3(1024), 0, st, a.blk, nb, ob->off, gerr, ob->ret);
      sg_outbound_sent o = *sent;
      TimedLaunch tl(ctx, "out_compact", 0.0);
      hipLaunchKernelGGL(k_out_compact, dim3(nb), dim3(256), 0, st, H, ob->start, ob->head, ob->rflags, ob->host_ip,
                         ob->ring, ob->cap, fwd_time, n_packets, ob->off, o);
    } else {
      hipLaunchKernelGGL(k_codel_reduce, dim3(1), dim3(1024), 0, st, a.blk, nb, gerr, ob->ret);
    }
    SG_CHECK_LAUNCH();
    SG_HIP(hipStreamSynchronize(st));
    const volatile unsigned long long* r = ob->ret;
    const uint64_t err = r[1];
    if (err & E_UNSORTED) throw Error(SG_ERR_UNSORTED, "sends must be grouped by ascending host");
    if (err & E_HOST) throw Error(SG_ERR_INVALID_ARG, "send host out of range");
    if (err & E_ORDER)
      throw Error(SG_ERR_UNSORTED, "a host's sends must come in execution order (time; Packet events, then "
                                   "Local ones by creation time and id)");
    if (err & E_FULL) throw Error(SG_ERR_CAPACITY, "an interface queue outgrew its ring (raise ring_cap)");
    if (err & E_PKT) throw Error(SG_ERR_INVALID_ARG, "packet id >= n_packets");
    if (err & E_WINDOW) throw Error(SG_ERR_INVALID_ARG, "a send is at or after window_end");
    const uint64_t ns = r[0];
    if (n_sent) *n_sent = (uint32_t)ns;
    if (sent && ns > sent->cap) throw Error(SG_ERR_CAPACITY, "the sent batch exceeds sent->cap");
  });
}

int32_t sg_outbound_get_state(sg_outbound* ob, sg_outbound_queue_state* o, sg_inbound_relay_state* rl) {
  if (!ob) return SG_ERR_INVALID_ARG;
  return sg::guarded(ob->ctx, [&] {
    const size_t n = ob->n, r = n * ob->cap;
    hipStream_t st = ob->ctx->stream;
    if (o) {
      struct { void* h; const void* d; size_t b; } cp[] = {{o->head, ob->head, n * 4}, {o->tail, ob->tail, n * 4}};
      for (auto& c : cp)
        if (c.h && c.b) SG_HIP(hipMemcpyAsync(c.h, c.d, c.b, hipMemcpyDeviceToHost, st));
    }
    if (rl) {
      struct { void* h; const void* d; size_t b; } cp[] = {
          {rl->flags, ob->rflags, n}, {rl->task_time, ob->task_time, n * 8}, {rl->tb_capacity, ob->tb_cap, n * 8},
          {rl->tb_balance, ob->tb_bal, n * 8}, {rl->tb_increment, ob->tb_inc, n * 8},
          {rl->tb_last_refill, ob->tb_last, n * 8}, {rl->task_event_id, ob->task_id, n * 8},
          {rl->task_created_ns, ob->task_born, n * 8}};
      for (auto& c : cp)
        if (c.h && c.b) SG_HIP(hipMemcpyAsync(c.h, c.d, c.b, hipMemcpyDeviceToHost, st));
    }
    std::vector<uint4> ring(o ? r : 0);
    if (o && r) SG_HIP(hipMemcpyAsync(ring.data(), ob->ring, r * 16, hipMemcpyDeviceToHost, st));
    SG_HIP(hipStreamSynchronize(st));
    if (o)
      for (size_t i = 0; i < r; i++) {
        if (o->ring_packet) o->ring_packet[i] = ring[i].x;
        if (o->ring_len) o->ring_len[i] = ring[i].y;
        if (o->ring_dst) o->ring_dst[i] = ring[i].z;
        if (o->ring_payload_len) o->ring_payload_len[i] = ring[i].w;
      }
    // the relay's cached packet is the ring slot at head - 1 (no separate fields)
    if (rl && (rl->cached_packet || rl->cached_len)) {
      std::vector<uint32_t> head(n);
      std::vector<uint8_t> fl(n);
      SG_HIP(hipMemcpy(head.data(), ob->head, n * 4, hipMemcpyDeviceToHost));
      SG_HIP(hipMemcpy(fl.data(), ob->rflags, n, hipMemcpyDeviceToHost));
      for (size_t h = 0; h < n; h++) {
        uint4 rec = make_uint4(0, 0, 0, 0);
        if (fl[h] & sg::R_CACHED)
          SG_HIP(hipMemcpy(&rec, ob->ring + h * ob->cap + ((head[h] - 1) & (ob->cap - 1)), 16, hipMemcpyDeviceToHost));
        if (rl->cached_packet) rl->cached_packet[h] = rec.x;
        if (rl->cached_len) rl->cached_len[h] = rec.y;
      }
    }
  });
}

}  // extern "C"
