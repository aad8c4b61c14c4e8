// sg_sssp.hip -- per-source shortest paths with the distance row resident in LDS.
//
// Replaces, for graphs whose node count fits a CU's LDS (about 11k nodes), the
// per-source petgraph::algo::dijkstra of NetworkGraph::compute_shortest_paths
// (graph/mod.rs:190-208).  One workgroup owns one source row: its keys
// key[v] = (latency u32 << 32) | bits(loss) live in LDS for the whole search,
// the graph's out-arcs are read from L2 (one 12-B record per relaxation), and
// the finished row is written straight into the caller's row-major table.
//
// Why not the batched-source slab kernel (sg_routing.hip k_relax_w2) here: a
// 64-source batch gathers whole 512-B rows, and Bellman-Ford re-gathers a row
// whenever any of its 64 sources improved it -- about 10x the n_used * arcs
// relaxations of Dijkstra at C3.  A per-source search relaxes only what its own
// frontier improved, and with the near/far bucket order below it does about
// 1.1-1.3x Dijkstra's relaxations.
//
// Exactness.  Edge latency >= 1 ns (graph/mod.rs:105-107) and the f32 loss fold
// is monotone, so petgraph's Dijkstra result is the unique fixed point of the
// source-rooted relaxation key[v] = min(key[v], key[u] (+) w(u, v)) with the
// edge applied on the right (sg_device.h relax32); any relaxation order reaches
// it.  LDS 64-bit atomic min keeps each (latency, loss) update whole.  Keys whose
// latency saturates at LAT32_SAT (>= 4.29 s, or unreachable) are never
// propagated and flag the row for the wide kernel (sg_routing.hip run_wide), as
// in the slab kernel.
//
// Work order: an asynchronous work queue per workgroup, with delta-stepping
// buckets (bucket width `delta`; one workgroup barrier per bucket, none per hop).
//   * dirty[v] (LDS bitmap) is set when key[v] improves and cleared when v is
//     popped.  A node becomes dirty once per improvement episode; an improvement
//     that makes it dirty with latency below `split` also appends it to the
//     queue, so the queue never holds a node twice.
//   * The queue is an LDS ring of u16 node ids with head / tail counters.  A
//     wave claims up to 64 entries (CAS on head), relaxes their out-arcs and
//     appends what it improved (add on tail, then the slot writes; a popped slot
//     not yet written reads as EMPTY and is waited for).  `busy` counts the
//     waves holding claimed entries; head and busy share one 64-bit LDS word,
//     so a claim is one CAS and a failed claim attempt changes nothing.
//   * Quiescence (busy == 0 and head == tail, read in that order) is stable: no
//     entry appears without a busy wave.  Every wave then meets at a barrier;
//     the dirty nodes left are those at or beyond `split`.  split = (smallest
//     dirty latency) + delta, the dirty nodes below it are queued, and the
//     waves go on.  No dirty node left: the search is done.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "sg_device.h"
#include "sg_internal.h"

namespace sg {

constexpr int SSSP_THREADS = 1024;
constexpr int SSSP_WAVES = SSSP_THREADS / 64;
constexpr int SSSP_K = 4;  // arc chunks (64 slots each) a wave handles at once
// static LDS of k_sssp_lds: ctl[8] + red[SSSP_WAVES] (u32), own[SSSP_WAVES][64 * SSSP_K] (u8)
constexpr size_t SSSP_STATIC_LDS = 4 * (8 + SSSP_WAVES) + 16 + SSSP_WAVES * 64 * SSSP_K;
constexpr size_t LDS_PER_CU = 160 * 1024;

// Inclusive scans across a wave64 with DPP (row shifts, then the row broadcasts
// of lanes 15 and 31): sum and max of u32.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false));
  return v;
}

// LDS bitmap updates.  Relaxed: a wave's LDS operations reach the LDS in issue
// order, and the order that matters (min on key[v], then the dirty bit; the
// dirty clear, then the key read) is kept by a control dependence and by a
// compiler fence.  A workgroup-scope acquire/release would also drain every
// outstanding global load (vmcnt(0)) on gfx950.
__device__ __forceinline__ uint32_t lds_fetch_or(uint32_t* p, uint32_t m) {
  return __hip_atomic_fetch_or(p, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_clear_bits(uint32_t* p, uint32_t m) {
  (void)__hip_atomic_fetch_and(p, ~m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Append the flagged lanes' node ids to an LDS list (one counter add per wave).
__device__ __forceinline__ void wave_append(bool flag, uint32_t node, uint16_t* list, uint32_t* counter,
                                            int lane) {
  const uint64_t m = __ballot(flag);
  if (!m) return;
  const int leader = __ffsll((unsigned long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
  base = __shfl(base, leader);
  if (flag) list[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = (uint16_t)node;
}

// Queue capacity: a power of two >= n + 1024.  At most n nodes are queued (one
// entry per dirty node) and at most 16 waves x 64 claimed slots are still being
// read, so a slot is never reused while its last entry is unread.
__host__ __device__ inline uint32_t sssp_ring_cap(uint32_t n) {
  uint32_t c = 1024;
  while (c < n + 1024) c <<= 1;
  return c;
}
constexpr uint16_t RING_EMPTY = 0xFFFF;

// LDS bytes the kernel needs for n nodes (dynamic part).
size_t sssp_lds_bytes(uint32_t n) {
  const size_t words = (n + 31) / 32;
  return (size_t)n * 8 + words * 4 + (size_t)sssp_ring_cap(n) * 2;
}

// One workgroup per source row i in [row_begin, row_end): source used[i].
// out_arc: 3 u32 per out-arc (destination, latency clamped to LAT32_SAT,
// bits(1f32 - loss)), grouped by tail node (out_off).
template <bool COUNT>
__global__ void __launch_bounds__(SSSP_THREADS)
    k_sssp_lds(const uint32_t* __restrict__ out_off, const uint32_t* __restrict__ out_arc, uint32_t n,
               uint32_t n_arcs, const uint32_t* __restrict__ used, uint32_t n_used, uint32_t row_begin,
               uint32_t out_row0, const uint32_t* __restrict__ self_edge, const uint64_t* __restrict__ e_lat,
               const float* __restrict__ e_loss, uint64_t* __restrict__ out_lat, float* __restrict__ out_loss,
               uint32_t* __restrict__ sat_row, uint32_t delta, int vec_out, unsigned long long* __restrict__ work,
               unsigned long long* __restrict__ diag) {
  extern __shared__ __align__(16) unsigned char smem[];
  const uint32_t W = (n + 31) / 32;
  const uint32_t cap = sssp_ring_cap(n), cmask = cap - 1;
  uint64_t* key = (uint64_t*)smem;
  uint32_t* dirty = (uint32_t*)(key + n);
  uint16_t* ring = (uint16_t*)(dirty + W);
  __shared__ uint32_t ctl[8];  // TAIL
  constexpr int TAIL = 1;
  // (head << 32) | busy in one word: a claim advances head and counts its wave
  // busy in one CAS, so a failed claim attempt never touches busy
  __shared__ unsigned long long hb;
  __shared__ uint8_t own[SSSP_WAVES][64 * SSSP_K];
  __shared__ uint32_t red[SSSP_WAVES];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // COUNT diagnostics of the first 4096 rows: cycle stamps, pops, bucket advances, relaxations
  const bool dg = COUNT && diag && blockIdx.x < 4096 && tid == 0;
  const unsigned long long c_start = dg ? clock64() : 0;
  uint32_t n_adv = 0, n_pops = 0;
  const uint32_t row = row_begin + blockIdx.x;
  const uint32_t src = used[row];
  for (uint32_t v = tid; v < n; v += SSSP_THREADS) key[v] = KEY_INF;
  for (uint32_t w = tid; w < W; w += SSSP_THREADS) dirty[w] = 0;
  for (uint32_t i = tid; i < cap; i += SSSP_THREADS) ring[i] = RING_EMPTY;
  for (int i = tid; i < SSSP_WAVES * 64 * SSSP_K; i += SSSP_THREADS) (&own[0][0])[i] = 0;
  if (tid < 8) ctl[tid] = 0;
  if (tid == 0) hb = 0;
  __syncthreads();
  if (tid == 0) {
    key[src] = 0;  // PathProperties::default()
    dirty[src >> 5] = 1u << (src & 31);
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
  bool gave_up = false;
  uint8_t* ow = own[wv];
  const uint64_t lt = (1ull << lane) - 1;
  // spin budget per wave (sleeps of ~64 cycles): a safety valve against a
  // queue bug, never reached by a correct search; past it the wave leaves and
  // the row goes to the wide kernel
  uint32_t spins = 0;
  constexpr uint32_t SPIN_MAX = 1u << 22;
  auto ld = [](uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
  __syncthreads();

  for (;;) {
    // ---- claim up to 64 queued entries
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
    if (!k) {
      uint32_t q = 0;
      if (lane == 0) {
        const unsigned long long w = __hip_atomic_load(&hb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);  // (head, busy) before tail (see header)
        q = (w & 0xFFFFFFFFull) == 0 && (uint32_t)(w >> 32) == ld(&ctl[TAIL]);
      }
      if (!__builtin_amdgcn_readfirstlane(q)) {
        if (++spins > SPIN_MAX) {
          gave_up = true;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
        continue;
      }
      // ---- quiescent: every wave is here.  Next bucket, or done.
      __syncthreads();
      uint32_t m = LAT32_SAT;
      for (uint32_t w = tid; w < W; w += SSSP_THREADS) {
        uint32_t bits = dirty[w];
        while (bits) {
          const uint32_t v = w * 32 + (uint32_t)__builtin_ctz(bits);
          bits &= bits - 1;
          m = min(m, key_lat(key[v]));
        }
      }
      for (int d = 32; d > 0; d >>= 1) m = min(m, (uint32_t)__shfl_xor(m, d));
      if (lane == 0) red[wv] = m;
      __syncthreads();
      m = red[0];
      for (int w = 1; w < SSSP_WAVES; w++) m = min(m, red[w]);
      if (m == LAT32_SAT) break;  // nothing dirty (saturated keys are never marked dirty)
      if (++n_adv > max_adv) {
        gave_up = true;
        break;
      }
      split = m + delta >= m ? min(m + delta, LAT32_SAT) : LAT32_SAT;
      for (uint32_t w0 = wv * 64; w0 < W; w0 += SSSP_THREADS) {  // queue the dirty nodes below split
        const uint32_t w = w0 + lane;
        uint32_t bits = w < W ? dirty[w] : 0u;
        for (;;) {
          const bool has = bits != 0;
          if (!__ballot(has)) break;
          const uint32_t v = has ? w * 32 + (uint32_t)__builtin_ctz(bits) : 0u;
          bits &= bits - 1;
          const bool q2 = has && key_lat(key[v]) < split;
          const uint64_t mq = __ballot(q2);
          if (mq) {
            uint32_t b = 0;
            if (lane == 0) b = atomicAdd(&ctl[TAIL], (uint32_t)__popcll(mq));
            b = __builtin_amdgcn_readfirstlane(b);
            if (q2) ring[(b + (uint32_t)__popcll(mq & lt)) & cmask] = (uint16_t)v;
          }
        }
      }
      __syncthreads();
      continue;
    }
    if (COUNT) n_pops++;
    // ---- pop the claimed entries (a slot claimed before its writer stored it reads EMPTY)
    const bool on = lane < (int)k;
    uint32_t u = 0, a0 = 0, a1 = 0;
    uint64_t ku = 0;
    bool stuck = false;
    if (on) {
      volatile uint16_t* slot = &ring[(h + lane) & cmask];
      uint16_t x;
      uint32_t sp = 0;
      while ((x = *slot) == RING_EMPTY && ++sp < SPIN_MAX) __builtin_amdgcn_s_sleep(0);
      stuck = x == RING_EMPTY;
      *slot = RING_EMPTY;
      u = stuck ? src : x;
      a0 = out_off[u];
      a1 = out_off[u + 1];
      lds_clear_bits(&dirty[u >> 5], 1u << (u & 31));  // before the key read (see header)
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      ku = key[u];
    }
    if (__any(stuck)) {
      if (lane == 0) atomicSub(&hb, 1ull);
      gave_up = true;
      break;
    }
    const uint32_t deg = a1 - a0;
    const uint32_t incl = wave_incl_sum(deg);
    const uint32_t base = incl - deg;
    const uint32_t T = __builtin_amdgcn_readlane(incl, 63);
    if (COUNT) n_rel += T;
    uint32_t carry = 0;  // 1 + the owner lane of the previous slot
    // NK chunks of 64 slots, straight-line (no per-chunk branch: a branch join
    // would make the compiler drain every load before the next is issued)
    auto step = [&](uint32_t t0, auto nk_c) {
      constexpr int NK = decltype(nk_c)::value;
      // owner lane of each slot: heads scatter 1 + their lane at their first slot, a max-scan fills the rest
      if (deg && base >= t0 && base - t0 < 64u * NK) ow[base - t0] = (uint8_t)(lane + 1);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      uint32_t v[NK], lat[NK], om[NK], o[NK];
      uint64_t cand[NK];
      bool valid[NK], imp[NK], app[NK];
#pragma unroll
      for (int c = 0; c < NK; c++) {
        const uint32_t hd = ow[c * 64 + lane];
        ow[c * 64 + lane] = 0;
        const uint32_t m = max(wave_incl_max(hd), carry);
        carry = __builtin_amdgcn_readlane(m, 63);
        o[c] = m - 1;
      }
#pragma unroll
      for (int c = 0; c < NK; c++) {
        const uint32_t sl = t0 + c * 64 + lane;
        valid[c] = sl < T;
        const uint32_t a = __shfl(a0, (int)o[c]) + sl - __shfl(base, (int)o[c]);
        const auto r = __builtin_amdgcn_raw_buffer_load_b96(arcs, valid[c] ? a * 12u : 0x80000000u, 0, 0);
        v[c] = r[0];
        lat[c] = r[1];
        om[c] = r[2];
      }
#pragma unroll
      for (int c = 0; c < NK; c++) {
        const uint32_t klo = __shfl((uint32_t)ku, (int)o[c]), khi = __shfl((uint32_t)(ku >> 32), (int)o[c]);
        cand[c] = relax32(((uint64_t)khi << 32) | klo, lat[c], __uint_as_float(om[c]));
        // a saturated key is never propagated (see header); an invalid slot offers KEY_INF
        if (!valid[c] || key_lat(cand[c]) == LAT32_SAT) cand[c] = KEY_INF;
      }
#pragma unroll
      for (int c = 0; c < NK; c++) {
        const uint64_t old = __hip_atomic_fetch_min((unsigned long long*)&key[valid[c] ? v[c] : 0],
                                                    (unsigned long long)cand[c], __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP);
        imp[c] = cand[c] < old;
      }
      uint32_t tot = 0;
      uint64_t mq[NK];
#pragma unroll
      for (int c = 0; c < NK; c++) {
        app[c] = false;
        if (imp[c]) {  // issued after the min returned (control dependence): see header
          const uint32_t bit = 1u << (v[c] & 31);
          app[c] = !(lds_fetch_or(&dirty[v[c] >> 5], bit) & bit) && key_lat(cand[c]) < split;
        }
        mq[c] = __ballot(app[c]);
        tot += (uint32_t)__popcll(mq[c]);
      }
      if (tot) {
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(&ctl[TAIL], tot);
        b = __builtin_amdgcn_readfirstlane(b);
#pragma unroll
        for (int c = 0; c < NK; c++) {
          if (app[c]) ring[(b + (uint32_t)__popcll(mq[c] & lt)) & cmask] = (uint16_t)v[c];
          b += (uint32_t)__popcll(mq[c]);
        }
      }
    };
    for (uint32_t t0 = 0; t0 < T; t0 += 64 * SSSP_K) {
      if (T - t0 > 64) step(t0, std::integral_constant<int, SSSP_K>{});
      else step(t0, std::integral_constant<int, 1>{});
    }
    // release the claim after this wave's appends (LDS keeps a wave's operations in order)
    if (lane == 0) atomicSub(&hb, 1ull);
  }
  if (COUNT && lane == 0 && n_rel) atomicAdd(&work[blockIdx.x & 63], (unsigned long long)n_rel);
  if (COUNT && diag && blockIdx.x < 4096 && lane == 0) {
    if (n_rel) atomicAdd(&diag[blockIdx.x * 8 + 4], (unsigned long long)n_rel);
    if (n_pops) atomicAdd(&diag[blockIdx.x * 8 + 2], (unsigned long long)n_pops);
  }
  const unsigned long long c_search = dg ? clock64() : 0;

  // ---- write the row: columns in used order, diagonal = the raw self-loop (graph/mod.rs:210-217)
  const size_t orow = (size_t)(row - out_row0) * n_used;
  bool sat = gave_up;
  auto entry = [&](uint32_t j, uint64_t& l, float& f) {
    if (j == row) {
      const uint32_t e = self_edge[used[j]];
      l = e_lat[e];
      f = e_loss[e];
    } else {
      const uint64_t k = key[used[j]];
      sat |= key_lat(k) == LAT32_SAT;
      l = key_lat(k);
      f = __uint_as_float(key_loss_bits(k));
    }
  };
  if (vec_out) {  // n_used % 4 == 0, 16-B aligned rows: 16-B nontemporal stores
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    for (uint32_t j = tid * 4; j < n_used; j += SSSP_THREADS * 4) {
      uint64_t l0, l1, l2, l3;
      float f0, f1, f2, f3;
      entry(j, l0, f0);
      entry(j + 1, l1, f1);
      entry(j + 2, l2, f2);
      entry(j + 3, l3, f3);
      __builtin_nontemporal_store((u64x2){l0, l1}, (u64x2*)&out_lat[orow + j]);
      __builtin_nontemporal_store((u64x2){l2, l3}, (u64x2*)&out_lat[orow + j + 2]);
      __builtin_nontemporal_store((f32x4){f0, f1, f2, f3}, (f32x4*)&out_loss[orow + j]);
    }
  } else {
    for (uint32_t j = tid; j < n_used; j += SSSP_THREADS) {
      uint64_t l;
      float f;
      entry(j, l, f);
      out_lat[orow + j] = l;
      out_loss[orow + j] = f;
    }
  }
  if (__any(sat) && lane == 0) sat_row[blockIdx.x] = 1u;
  if (dg) {
    diag[blockIdx.x * 8 + 0] = c_search - c_start;
    diag[blockIdx.x * 8 + 1] = clock64() - c_search;
    diag[blockIdx.x * 8 + 3] = n_adv;
  }
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
                     unsigned long long* diag) {
  const size_t lds = sssp_lds_bytes(n);
  if (!sssp_lds_fits(n)) throw Error(SG_ERR_INVALID_ARG, "graph too large for the LDS-resident search");
  if ((uint64_t)n_arcs * 12 >= (1ull << 31)) throw Error(SG_ERR_INVALID_ARG, "too many arcs for 32-bit offsets");
  const int vec = n_used % 4 == 0 && ((uintptr_t)out_lat & 15) == 0 && ((uintptr_t)out_loss & 15) == 0;
  const uint32_t rows = row_end - row_begin;
  if (!rows) return;
  if (work) {
    SG_HIP(hipFuncSetAttribute((const void*)k_sssp_lds<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(LDS_PER_CU - SSSP_STATIC_LDS)));
    hipLaunchKernelGGL(k_sssp_lds<true>, dim3(rows), dim3(SSSP_THREADS), lds, ctx->stream, out_off, out_arc, n,
                       n_arcs, d_used, n_used, row_begin, row_begin, self_edge, e_lat, e_loss, out_lat, out_loss,
                       sat_row, delta, vec, work, diag);
  } else {
    SG_HIP(hipFuncSetAttribute((const void*)k_sssp_lds<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(LDS_PER_CU - SSSP_STATIC_LDS)));
    hipLaunchKernelGGL(k_sssp_lds<false>, dim3(rows), dim3(SSSP_THREADS), lds, ctx->stream, out_off, out_arc, n,
                       n_arcs, d_used, n_used, row_begin, row_begin, self_edge, e_lat, e_loss, out_lat, out_loss,
                       sat_row, delta, vec, work, diag);
  }
  SG_CHECK_LAUNCH();
}

}  // namespace sg
