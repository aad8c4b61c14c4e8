// sg_dense.hip -- per-source shortest paths on dense graphs (C2: the 1,200-node
// complete graph of docs/network_graph_overview.md:58-63).
//
// Replaces, for graphs of at most DENSE_MAX nodes whose mean out-degree is past
// the sparse searches' range, the per-source petgraph::algo::dijkstra of
// NetworkGraph::compute_shortest_paths (graph/mod.rs:190-208).
//
// One workgroup per source row, its keys in LDS.  Two searches: the lazy search
// (k_sssp_dense_lazy, the default since r6; see "Lazy relaxation" below), and the
// T-cut search described here (k_sssp_dense; SG_DENSE_LAZY=0, with seed rows).  Both
// settle nodes in rounds (Dijkstra with a width) and relax only the arcs that can
// still matter:
//
//  * Settling.  A round takes m = the smallest latency of the unsettled keys and
//    settles every unsettled v with key(v).lat < m + w_min (w_min = the smallest
//    arc latency, >= 1 ns by graph/mod.rs:105-107).  Such a key is final: any
//    other path to v leaves the settled set through an unsettled node x, so its
//    latency is at least key(x).lat + w_min >= m + w_min > key(v).lat -- larger
//    in the PathProperties order (latency first, graph/mod.rs:305-313).
//  * Pruning.  The round also takes T = the largest latency of the unsettled
//    keys (LAT32_SAT while any is unreached).  Keys only fall during the round, so
//    a candidate with latency > T improves no unsettled key, and no settled one
//    (those are below every later candidate).  Each node's out-arcs are sorted by
//    latency once per build (k_sort_arcs), so a settled row u is relaxed only up
//    to its first arc with key(u).lat + w > T.  On a complete graph with random
//    latencies that is a few percent of the row: Dijkstra's n^2 arc reads per
//    source shrink to the short arcs, which every source shares (they stay in L2).
//
// Relaxation is the 64-bit LDS atomic min of sg_sssp.hip on the packed key
// (latency << 32 | bits(loss)), whose integer order is the PathProperties order;
// the fold applies the edge on the right (sg_device.h relax32), so the result is
// the fixed point petgraph's Dijkstra returns (sg_sssp.hip header).  Parallel
// arcs need no merging: the worse one's candidate loses its atomic min.
//
// Keys saturate at LAT32_SAT like every 32-bit kernel: a saturated candidate is
// never offered, and a row with a saturated (unreachable or >= 4.29 s) key is
// flagged for the wide kernel (sg_routing.hip run_wide).
#include <algorithm>
#include <vector>

#include "sg_device.h"
#include "sg_internal.h"

namespace sg {

// threads per row of the unseeded launch (r8x A/B builds: 512 and 256 threads measured 0.317-0.321
// and 0.312-0.316 ms against 0.301-0.303 for 1024 at C2; the seeded launches: SG_DENSE_SEED_THREADS)
constexpr int DENSE_THREADS = 1024;
constexpr uint32_t DENSE_SCAP = 512;    // nodes settled per round at most (the rest wait a round)
constexpr uint32_t SORT_MAXDEG = 4096;  // out-degree sorted in one block's LDS; larger rows stay unsorted
#ifndef DN_G  // (A/B builds at C2, r8y: 1 row 0.320-0.323 ms, 3 rows 0.304-0.305, 4 rows 0.454-0.455, 2 rows 0.304-0.306)
#define DN_G 2
#endif
constexpr int DENSE_G = DN_G;           // settled rows a wave relaxes together (their loads in flight)
// Sorted-arc records of 12 B (b96 loads; DN_REC16 builds the 16-B records with a pad word of r04).
// A/B knobs (C2, r7h, `profiles/r05/ab_c2_dense_r7h.txt`): 12-B records 0.461-0.465 ms against
// 0.469-0.474 for 16 B; nt loads in a round whose cut is still open (a row's whole arc list, read
// once; DN_NT1, removed r6) 0.520; DN_NTOUT (nontemporal table stores) 0.470-0.472.
#ifndef DN_REC16
#define DN_REC12
#endif
#ifdef DN_REC12
constexpr uint32_t DN_W = 3;
#else
constexpr uint32_t DN_W = 4;
#endif

// Per node u: its out-arcs (out_arc, 3 u32 each: head, latency32, bits(1f32 - loss))
// sorted by latency into 12-B records {head, latency32, bits(om)} (16 B with a pad word
// under DN_REC16) at the same offsets; sorted[u] = 1, or 0 for a row past `cap` arcs (copied as is, never cut
// short).  Also the smallest arc latency (w_min).  One block per node; cap = the LDS
// array (a power of two >= n - 1, at most SORT_MAXDEG: parallel arcs can exceed it).
constexpr int SORT_THREADS = 1024;
__global__ void __launch_bounds__(SORT_THREADS) k_sort_arcs(const uint32_t* __restrict__ out_off,
                                                            const uint32_t* __restrict__ out_arc, uint32_t cap,
                                                            uint32_t* __restrict__ sa, uint8_t* __restrict__ sorted,
                                                            uint32_t* __restrict__ wmin) {
  extern __shared__ __align__(16) unsigned long long k[];  // [cap]
  __shared__ uint32_t s_lo[SORT_THREADS / 64];
  const uint32_t u = blockIdx.x, t = threadIdx.x;
  const uint32_t a0 = out_off[u], deg = out_off[u + 1] - a0;
  uint32_t lo = LAT32_SAT;
  if (deg > cap) {
    for (uint32_t i = t; i < deg; i += SORT_THREADS) {
      const uint32_t* r = out_arc + 3 * (size_t)(a0 + i);
      uint32_t* d = sa + DN_W * (size_t)(a0 + i);
      d[0] = r[0];
      d[1] = r[1];
      d[2] = r[2];
      if (DN_W == 4) d[3] = 0u;
      lo = min(lo, r[1]);
    }
    if (t == 0) sorted[u] = 0;
  } else {
    uint32_t M = 1;
    while (M < deg) M <<= 1;
    for (uint32_t i = t; i < M; i += SORT_THREADS) {
      const uint32_t l = i < deg ? out_arc[3 * (size_t)(a0 + i) + 1] : LAT32_SAT;
      k[i] = i < deg ? ((unsigned long long)l << 32) | i : ~0ull;
      lo = min(lo, l);
    }
    __syncthreads();
    for (uint32_t kk = 2; kk <= M; kk <<= 1)
      for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
        for (uint32_t i = t; i < M; i += SORT_THREADS) {
          const uint32_t l = i ^ j;
          if (l > i) {
            const unsigned long long x = k[i], y = k[l];
            if ((y < x) == ((i & kk) == 0)) {
              k[i] = y;
              k[l] = x;
            }
          }
        }
        __syncthreads();
      }
    for (uint32_t i = t; i < deg; i += SORT_THREADS) {
      const uint32_t* r = out_arc + 3 * (size_t)(a0 + (uint32_t)(k[i] & 0xFFFFFFFFu));
      uint32_t* d = sa + DN_W * (size_t)(a0 + i);
      d[0] = r[0];
      d[1] = r[1];
      d[2] = r[2];
      if (DN_W == 4) d[3] = 0u;
    }
    if (t == 0) sorted[u] = 1;
  }
  for (int d = 32; d > 0; d >>= 1) lo = min(lo, (uint32_t)__shfl_xor(lo, d, 64));
  if ((t & 63) == 0) s_lo[t >> 6] = lo;
  __syncthreads();
  if (t == 0) {
    uint32_t m = LAT32_SAT;
    for (int w = 0; w < SORT_THREADS / 64; w++) m = min(m, s_lo[w]);
    if (m != LAT32_SAT) atomicMin(wmin, m);
  }
}

// ---- write a row: columns in used order, diagonal = the raw self-loop (graph/mod.rs:210-217);
// a saturated off-diagonal key flags the row for the wide kernel
template <int TH>
__device__ __forceinline__ void dense_write_row(const unsigned long long* key, uint32_t src, uint32_t row,
                                                const uint32_t* __restrict__ used, uint32_t n_used,
                                                const uint32_t* __restrict__ self_edge,
                                                const uint64_t* __restrict__ e_lat, const float* __restrict__ e_loss,
                                                uint64_t* __restrict__ olat, float* __restrict__ oloss,
                                                uint32_t* __restrict__ sat_flag) {
  bool sat = false;
  const uint32_t de = self_edge[src];
  for (uint32_t jj = threadIdx.x; jj < n_used; jj += TH) {
    const uint32_t v = used[jj];
    const unsigned long long k = key[v];
    const bool diag = jj == row;
    sat |= !diag && key_lat(k) == LAT32_SAT;
#ifdef DN_NTOUT
    __builtin_nontemporal_store(diag ? e_lat[de] : (uint64_t)key_lat(k), &olat[jj]);
    __builtin_nontemporal_store(diag ? e_loss[de] : __uint_as_float(key_loss_bits(k)), &oloss[jj]);
#else
    olat[jj] = diag ? e_lat[de] : (uint64_t)key_lat(k);
    oloss[jj] = diag ? e_loss[de] : __uint_as_float(key_loss_bits(k));
#endif
  }
  // the row's flag written whatever its value (every row is one block's), so no fill precedes a build
  const int any = __syncthreads_or(sat ? 1 : 0);
  if (threadIdx.x == 0) *sat_flag = any ? 1u : 0u;
}

// Seeded rows (SG_DENSE_SEED, launch_sssp_dense): the block's rows run in levels, one launch
// each.  The first computes its rows from scratch; every launch but the last stamps its
// sources in `mark` (gen << 16 | row within the block); a later launch starts each row's keys
// at the bounds of its nearest out-neighbour stamped by an EARLIER launch (stamp generation in
// [gen_lo, gen): finished rows, never one of its own), so the cut T is tight from the first
// round instead of the row's longest arc.
enum : uint32_t { DENSE_SEED_MARK = 1, DENSE_SEED_USE = 2 };
struct DenseSeed {
  uint32_t mode, gen_lo, gen, row0;  // row0: the block's first row (the stamps' row origin)
  uint32_t* mark;                    // [n] per node
  const uint64_t* lat;               // the block's rows of the table
};

template <int TH, uint32_t SW>
__global__ void __launch_bounds__(TH) k_sssp_dense(const uint32_t* __restrict__ out_off,
                                                              const uint32_t* __restrict__ sa,
                                                              const uint8_t* __restrict__ sorted, uint32_t n,
                                                              uint32_t n_arcs, const uint32_t* __restrict__ wmin_p,
                                                              const uint32_t* __restrict__ used, uint32_t n_used,
                                                              uint32_t row_begin, const uint32_t* __restrict__ self_edge,
                                                              const uint64_t* __restrict__ e_lat,
                                                              const float* __restrict__ e_loss,
                                                              uint64_t* __restrict__ out_lat,
                                                              float* __restrict__ out_loss,
                                                              uint32_t* __restrict__ sat_row,
                                                              unsigned long long* __restrict__ work,
                                                              uint32_t split_below, DenseSeed sd) {
  constexpr int TW = TH / 64;
  extern __shared__ __align__(16) unsigned char smem[];
  unsigned long long* key = (unsigned long long*)smem;        // [n]
  uint32_t* settled = (uint32_t*)(key + n);                   // [ceil(n / 32)] bitmap
  const uint32_t nbw = (n + 31) / 32;
  uint32_t* s_node = settled + ((nbw + 1) & ~1u);             // [DENSE_SCAP] this round's settled nodes
  __shared__ uint32_t s_cnt;
  __shared__ uint32_t red_m[TW], red_t[TW];
  __shared__ uint32_t s_m, s_t, s_prow, s_pw;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t row = row_begin + blockIdx.x;
  const uint32_t src = used[row];
  const uint32_t wmin = *wmin_p;  // >= 1 (graph/mod.rs:105-107); LAT32_SAT: no arc at all
  for (uint32_t v = t; v < n; v += TH) key[v] = v == src ? 0ull : KEY_INF;  // default() at the source
  for (uint32_t i = t; i < nbw; i += TH) settled[i] = 0u;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)sa, 0, (int)0x7FFFFFFF, 0x00020000);
  unsigned long long n_rel = 0;
  if ((sd.mode & DENSE_SEED_MARK) && t == 0) sd.mark[src] = (sd.gen << 16) | (row - sd.row0);
  if (sd.mode & DENSE_SEED_USE) {
    // the seed row: the first (lightest, the arcs being sorted) out-arc s -> p to a row p of
    // the seed launch; its row bounds every key, d(s, v) <= w(s, p) + D[p][v]
    if (wv == 0) {
      uint32_t prow = ~0u, pw = 0;
      const uint32_t e = out_off[src + 1];
      for (uint32_t c = out_off[src]; c < e; c += 64) {
        const uint32_t i = c + lane;
        uint32_t h = src, l = 0, mk = 0;
        if (i < e) {
          h = sa[DN_W * (size_t)i];
          l = sa[DN_W * (size_t)i + 1];
          mk = sd.mark[h];
        }
        const uint64_t hit = __ballot(h != src && (mk >> 16) >= sd.gen_lo && (mk >> 16) < sd.gen);
        if (hit) {
          const int f = __builtin_ctzll(hit);
          prow = (uint32_t)__builtin_amdgcn_readlane((int)(mk & 0xFFFFu), f);
          pw = (uint32_t)__builtin_amdgcn_readlane((int)l, f);
          break;
        }
      }
      if (lane == 0) {
        s_prow = prow;
        s_pw = pw;
      }
    }
    __syncthreads();
    const uint32_t prow = s_prow, pw = s_pw;
    if (prow != ~0u) {
      // a bound key (UB + 1, loss 1.0) lies above every real path of latency <= UB, so the
      // node is settled only once a real candidate has replaced it (the settling argument of
      // the header needs keys >= the true value, which bounds are); it only tightens T
      const uint64_t* prw = sd.lat + (size_t)prow * n_used;
      const uint32_t pcol = sd.row0 + prow;
      for (uint32_t jj = t; jj < n_used; jj += TH) {
        const uint32_t v = used[jj];
        if (v == src) continue;
        const uint64_t b = (jj == pcol ? 0ull : prw[jj]) + pw + 1ull;
        if (b < LAT32_SAT) key[v] = (b << 32) | 0x3F800000ull;
      }
    }
  }
  __syncthreads();
  for (;;) {
    // the smallest and largest latency of the unsettled keys
    uint32_t m = LAT32_SAT, T = 0;
    for (uint32_t v = t; v < n; v += TH) {
      if (settled[v >> 5] >> (v & 31) & 1u) continue;
      const uint32_t l = key_lat(key[v]);
      m = min(m, l);
      T = max(T, l);
    }
    for (int d = 32; d > 0; d >>= 1) {
      m = min(m, (uint32_t)__shfl_xor(m, d, 64));
      T = max(T, (uint32_t)__shfl_xor(T, d, 64));
    }
    if (lane == 0) {
      red_m[wv] = m;
      red_t[wv] = T;
    }
    __syncthreads();
    if (t == 0) {
      uint32_t mm = LAT32_SAT, tt = 0;
      for (int k = 0; k < TW; k++) {
        mm = min(mm, red_m[k]);
        tt = max(tt, red_t[k]);
      }
      s_m = mm;
      s_t = tt;
      s_cnt = 0;
    }
    __syncthreads();
    m = s_m;
    T = s_t;
    if (m == LAT32_SAT) break;  // every key settled, or saturated (unreachable in 32 bits: the wide kernel)
    const uint32_t thr = m + wmin >= m ? m + wmin : LAT32_SAT;  // settle key.lat < thr
    for (uint32_t v0 = wv * 64; v0 < n; v0 += TH) {
      const uint32_t v = v0 + lane;
      const bool s = v < n && !(settled[v >> 5] >> (v & 31) & 1u) && key_lat(key[v]) < thr;
      const uint64_t bal = __ballot(s);
      if (!bal) continue;
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(&s_cnt, (uint32_t)__popcll(bal));
      base = __builtin_amdgcn_readfirstlane(base);
      const uint32_t pos = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
      if (s && pos < DENSE_SCAP) {  // past the cap a node waits a round (it stays below the threshold)
        s_node[pos] = v;
        atomicOr(&settled[v >> 5], 1u << (v & 31));
      }
    }
    __syncthreads();
    const uint32_t ns = min(s_cnt, DENSE_SCAP);
    // Relax: a wave takes DENSE_G settled rows at a time, 64 arcs per row and step, and
    // stops a row at its first arc past T (rows sorted by latency); keys are final for
    // the settled rows (their (lat, loss) read once here, unchanged during the round).
    // A round with few settled rows (the first ones, whose cut is still near the longest arc:
    // whole rows) splits each row over TW / ns waves, which take its 64-arc chunks in
    // turn -- the row's loads in flight side by side instead of one chunk after the other.
    if (ns < split_below) {
      const uint32_t per = TW / ns, r = wv % ns, p = wv / ns;
      if (p < per) {
        const uint32_t u = s_node[r];
        const uint32_t e = out_off[u + 1];
        const uint64_t kuv = key[u];
        const bool cutr = sorted[u];
        const uint32_t budget = T - min(T, key_lat(kuv));
        for (uint32_t c0 = out_off[u] + 64 * p; c0 < e; c0 += 64 * per) {
          const uint32_t i = c0 + lane;
          const uint32_t off = i < e ? i * (4u * DN_W) : 0x80000000u;
#ifdef DN_REC12
          const auto x = __builtin_amdgcn_raw_buffer_load_b96(ra, off, 0, 0);
#else
          const auto x = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0);
#endif
          const bool in = i < e && (!cutr || x[1] <= budget);
          const uint64_t cd = relax32(kuv, x[1], __uint_as_float(x[2]));
          const bool offer = in && key_lat(cd) != LAT32_SAT && !(settled[x[0] >> 5] >> (x[0] & 31) & 1u);
          if (offer) (void)__hip_atomic_fetch_min(&key[x[0]], (unsigned long long)cd, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_WORKGROUP);
          if (work) n_rel += __popcll(__ballot(in));
          if (!__builtin_amdgcn_readlane((int)in, 63)) break;  // the cut (or the row's end): later chunks are past it
        }
      }
      __syncthreads();
      continue;
    }
    // Lane groups of SW lanes: a wave relaxes DENSE_G * 64 / SW settled rows side by side, SW arcs
    // of each per step (SW < 64 for rows cut short: the seeded launches' settled rows have ~15
    // arcs under the cut, which a 64-lane step would load a quarter full)
    constexpr uint32_t NGR = 64 / SW;
    const uint32_t gl = lane % SW, gi = lane / SW;
    for (uint32_t s0 = wv * DENSE_G * NGR; s0 < ns; s0 += TW * DENSE_G * NGR) {
      uint32_t a[DENSE_G], e[DENSE_G], budget[DENSE_G];
      uint64_t ku[DENSE_G];
      bool cut[DENSE_G];
#pragma unroll
      for (int g = 0; g < DENSE_G; g++) {
        const uint32_t si = s0 + g * NGR + gi;
        const bool ok = si < ns;
        const uint32_t u = ok ? s_node[si] : 0u;
        a[g] = ok ? out_off[u] : 0u;
        e[g] = ok ? out_off[u + 1] : 0u;
        ku[g] = ok ? key[u] : KEY_INF;
        cut[g] = ok && sorted[u];
        budget[g] = T - min(T, key_lat(ku[g]));  // the latency budget of the row's arcs: key(u).lat + w <= T
      }
      bool live = true;
      while (live) {
        uint4 r[DENSE_G];
#pragma unroll
        for (int g = 0; g < DENSE_G; g++) {
          const uint32_t i = a[g] + gl;
          const uint32_t off = i < e[g] ? i * (4u * DN_W) : 0x80000000u;
#ifdef DN_REC12
          const auto x = __builtin_amdgcn_raw_buffer_load_b96(ra, off, 0, 0);
          r[g] = make_uint4(x[0], x[1], x[2], 0u);
#else
          const auto x = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0);
          r[g] = make_uint4(x[0], x[1], x[2], x[3]);
#endif
        }
        uint64_t more_any = 0;
#pragma unroll
        for (int g = 0; g < DENSE_G; g++) {
          const uint32_t i = a[g] + gl;
          const bool in = i < e[g] && (!cut[g] || r[g].y <= budget[g]);
          const uint64_t cd = relax32(ku[g], r[g].y, __uint_as_float(r[g].z));
          const bool offer = in && key_lat(cd) != LAT32_SAT && !(settled[r[g].x >> 5] >> (r[g].x & 31) & 1u);
          if (offer) (void)__hip_atomic_fetch_min(&key[r[g].x], (unsigned long long)cd, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_WORKGROUP);
          const uint64_t bin = __ballot(in);
          if (work) n_rel += __popcll(bin);
          // a row goes on while its group's last lane's arc is in range and within the budget
          const bool more = (bin >> (gi * SW + SW - 1) & 1u) && a[g] + SW < e[g];
          a[g] = more ? a[g] + SW : e[g];
          more_any |= __ballot(more);
        }
        live = more_any != 0;
      }
    }
    __syncthreads();
  }
  if (work && lane == 0 && n_rel) atomicAdd(&work[blockIdx.x & 63], n_rel);
  dense_write_row<TH>(key, src, row, used, n_used, self_edge, e_lat, e_loss, out_lat + (size_t)blockIdx.x * n_used,
                      out_loss + (size_t)blockIdx.x * n_used, sat_row + blockIdx.x);
}

// ---------------------------------------------------------------------------
// Lazy relaxation (SG_DENSE_LAZY; r6).  Rounds of settled nodes as above, but a settled row is
// not relaxed once up to the round's largest unsettled key T: it is relaxed up to the round's
// threshold only, and resumed in later rounds where it stopped (its arcs are sorted: ptr = the
// first arc not yet relaxed, nxt = that arc's latency, both in LDS).  A round, from
// m = the smallest unsettled key and me = the smallest key(u).lat + nxt[u] of the settled rows:
//   1. thr = min(m, me) + w_min (m + w_min after a round that settled nothing; me + a doubling
//      budget while no key below LAT32_SAT is unsettled); list the settled rows with
//      key(u).lat + nxt[u] < thr;
//   2. relax them, SW lanes per row, over their arcs with key(u).lat + w < thr, and record where
//      each stopped; m2 = min(m, the smallest latency offered to an unsettled node);
//   3. settle every unsettled v with key(v).lat < min(thr, m2 + w_min); the scan also gives the
//      next round's m and me.
// Step 3 is Dijkstra's rule: a path to v other than its key leaves the settled set over an arc
// not yet relaxed (latency >= thr, every arc below thr having been relaxed) or through an
// unsettled x != v (latency >= key(x).lat + w_min >= m2 + w_min).  Of two rounds in a row with m
// below LAT32_SAT one settles a node; a round without relaxes rows from me over a doubling
// budget -- so the search ends, when every node is settled or no key below LAT32_SAT is left unsettled and no
// settled row has an arc left whose candidate stays below it.  Each row relaxes only its arcs below the largest final key plus w_min: C2 ~11k arcs per
// source against ~88k under the T cut (~15k with seed rows), in one launch without seed rows.
// A row past the sort's `cap` (sorted[u] = 0, nxt = 0: listed at once) is relaxed whole.
#ifdef DN_PROF
// diagnostic build only (-DDN_PROF): per-phase wall-clock totals of the lazy search, 10-ns ticks:
// init, listing, relaxation, settling, write-out, rounds, rows listed, whole row
__device__ unsigned long long g_dn_prof[8];
#endif
template <int TH, uint32_t SW, int G, bool SPEC, bool RTN = false>
__global__ void __launch_bounds__(TH) k_sssp_dense_lazy(const uint32_t* __restrict__ out_off,
                                                        const uint32_t* __restrict__ sa,
                                                        const uint8_t* __restrict__ sorted, uint32_t n,
                                                        const uint32_t* __restrict__ wmin_p,
                                                        const uint32_t* __restrict__ used, uint32_t n_used,
                                                        uint32_t row_begin, const uint32_t* __restrict__ self_edge,
                                                        const uint64_t* __restrict__ e_lat,
                                                        const float* __restrict__ e_loss,
                                                        uint64_t* __restrict__ out_lat, float* __restrict__ out_loss,
                                                        uint32_t* __restrict__ sat_row,
                                                        unsigned long long* __restrict__ work) {
  constexpr int TW = TH / 64;
  constexpr uint32_t NGR = 64 / SW;  // rows per wave and step
  constexpr uint32_t UNSORTED = 0x80000000u;  // end[] flag (arc indices < 2^31: launch_sssp_dense)
  extern __shared__ __align__(16) unsigned char smem[];
  unsigned long long* key = (unsigned long long*)smem;  // [n]
  uint32_t* ptr = (uint32_t*)(key + n);                 // [n] the first arc not yet relaxed
  uint32_t* end = ptr + n;                              // [n] the row's end | UNSORTED
  uint32_t* nxt = end + n;                              // [n] ptr's latency (LAT32_SAT: none left)
  uint32_t* lst = nxt + n;                              // [n] this round's rows to relax
  uint32_t* settled = lst + n;                          // [ceil(n / 32)] bitmap
  const uint32_t nbw = (n + 31) / 32;
  __shared__ uint32_t s_cnt, s_mo, s_m, s_me, s_un, s_new;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t gl = lane % SW, gi = lane / SW;
  const uint32_t row = row_begin + blockIdx.x;
  const uint32_t src = used[row];
  const uint32_t wmin = *wmin_p;  // >= 1 (graph/mod.rs:105-107); LAT32_SAT: no arc at all
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)sa, 0, (int)0x7FFFFFFF, 0x00020000);
#ifdef DN_PROF
  const unsigned long long pt_start = wall_clock64();
#endif
  for (uint32_t v = t; v < n; v += TH) {
    key[v] = v == src ? 0ull : KEY_INF;  // default() at the source
    const uint32_t a0 = out_off[v], e0 = out_off[v + 1];
    const bool so = sorted[v];
    ptr[v] = a0;
    end[v] = e0 | (so ? 0u : UNSORTED);
    nxt[v] = a0 == e0 ? LAT32_SAT : !so ? 0u : sa[DN_W * (size_t)a0 + 1];
  }
  for (uint32_t i = t; i < nbw; i += TH) settled[i] = 0u;
  if (t == 0) s_cnt = 0;
  unsigned long long n_rel = 0;
  uint32_t m = 0, me = LAT32_SAT, un = 1;  // the source: the only key, unsettled
  uint32_t k_far = 0;   // rounds in a row with no unsettled key below LAT32_SAT (see thr below)
  uint32_t settled_any = 1;  // the last round settled a node
  __syncthreads();
#ifdef DN_PROF
  unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tq = wall_clock64(), t0q = tq;
  pt[0] = tq - pt_start;
#define DN_MARK(k) do { const unsigned long long q_ = wall_clock64(); pt[k] += q_ - tq; tq = q_; } while (0)
#else
#define DN_MARK(k) do {} while (0)
#endif
  for (;;) {
    const uint32_t base = min(m, me);
    // (uniform) every node settled, or nothing left below LAT32_SAT (unreachable or saturated
    // keys: the wide kernel's)
    if (!un || base == LAT32_SAT) break;
    // The relaxation threshold.  Any thr works for exactness (every arc below it is relaxed
    // before the settling rule uses it); it is chosen for progress.  With an unsettled key m:
    // thr = min(m, me) + w_min, or m + w_min after a round that settled nothing -- then the node
    // of key m2 <= m settles, so there are at most 2n such rounds.  With none (m = LAT32_SAT: the
    // nodes left are unreached so far), the rows' next arcs from me on are relaxed over a budget
    // that doubles each such round in a row: at most ~32 of them before the whole rest is
    // relaxed.  (thr = min(m, me) + w_min alone took one round per distinct candidate value on a
    // graph whose far nodes are reached over long arcs and a 1-ns w_min; m + w_min every round
    // cost C2 0.130 ms against 0.125.)
    uint32_t thr;
    if (m != LAT32_SAT) {
      const uint32_t b = settled_any ? base : m;
      thr = b + wmin >= b ? b + wmin : LAT32_SAT;
      k_far = 0;
    } else {
      const uint64_t x = (uint64_t)wmin << min(k_far, 32u);
      thr = (uint32_t)min((uint64_t)me + x, (uint64_t)LAT32_SAT);
      k_far++;
    }
    // 1. the settled rows with an arc below thr
    for (uint32_t v0 = wv * 64; v0 < n; v0 += TH) {
      const uint32_t v = v0 + lane;
      bool s = false;
      if (v < n && (settled[v >> 5] >> (v & 31) & 1u))
        s = __builtin_elementwise_add_sat(key_lat(key[v]), nxt[v]) < thr;
      const uint64_t bal = __ballot(s);
      if (!bal) continue;
      uint32_t b0 = 0;
      if (lane == 0) b0 = atomicAdd(&s_cnt, (uint32_t)__popcll(bal));
      b0 = __builtin_amdgcn_readfirstlane(b0);
      if (s) lst[b0 + (uint32_t)__popcll(bal & ((1ull << lane) - 1))] = v;
    }
    if (t == 0) {
      s_mo = m;
      s_m = LAT32_SAT;
      s_me = LAT32_SAT;
      s_un = 0;
      s_new = 0;
    }
    __syncthreads();
    const uint32_t nl = s_cnt;
    DN_MARK(1);
#ifdef DN_PROF
    pt[5] += 1;
    pt[6] += nl;
#endif
    // 2. relax them up to thr: SW lanes per row, G * NGR rows per wave side by side
    uint32_t mo = LAT32_SAT;
    for (uint32_t s0 = wv * G * NGR; s0 < nl; s0 += TW * G * NGR) {
      uint32_t a[G], e[G], budget[G], u[G];
      uint64_t ku[G];
#pragma unroll
      for (int g = 0; g < G; g++) {
        const uint32_t si = s0 + g * NGR + gi;
        const bool ok = si < nl;
        u[g] = ok ? lst[si] : 0u;
        a[g] = ok ? ptr[u[g]] : 0u;
        const uint32_t ed = ok ? end[u[g]] : 0u;
        e[g] = ed & ~UNSORTED;
        ku[g] = ok ? key[u[g]] : KEY_INF;
        // arcs with key(u).lat + w < thr (key(u).lat + nxt[u] < thr: the budget is >= nxt[u]);
        // an unsorted row whole
        budget[g] = !ok ? 0u : (ed & UNSORTED) ? LAT32_SAT : thr - 1u - key_lat(ku[g]);
      }
      bool live = true;
      while (live) {
        uint4 r[G];
#pragma unroll
        for (int g = 0; g < G; g++) {
          const uint32_t i = a[g] + gl;
          const uint32_t off = i < e[g] ? i * (4u * DN_W) : 0x80000000u;
#ifdef DN_REC12
          const auto x = __builtin_amdgcn_raw_buffer_load_b96(ra, off, 0, 0);
          r[g] = make_uint4(x[0], x[1], x[2], 0u);
#else
          const auto x = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0);
          r[g] = make_uint4(x[0], x[1], x[2], x[3]);
#endif
        }
        uint64_t more_any = 0;
#pragma unroll
        for (int g = 0; g < G; g++) {
          const uint32_t i = a[g] + gl;
          // SPEC: the whole chunk once it is loaded (arcs past thr are real paths too: candidates
          // that only come early), and the next chunk while this one's last arc is within budget
          const bool in = i < e[g] && (SPEC || r[g].y <= budget[g]);
          const uint64_t cd = relax32(ku[g], r[g].y, __uint_as_float(r[g].z));
          if (RTN) {
            // no settled-bit read ahead of the atomic: a settled node's key is final, so no real
            // path's candidate lowers it; the returned key tells an improvement (an unsettled
            // node), which alone may lower m
            if (in && key_lat(cd) != LAT32_SAT) {
              const unsigned long long old = __hip_atomic_fetch_min(&key[r[g].x], (unsigned long long)cd,
                                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              if (cd < old) mo = min(mo, key_lat(cd));
            }
          } else {
            const bool offer = in && key_lat(cd) != LAT32_SAT && !(settled[r[g].x >> 5] >> (r[g].x & 31) & 1u);
            if (offer) {
              (void)__hip_atomic_fetch_min(&key[r[g].x], (unsigned long long)cd, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
              mo = min(mo, key_lat(cd));
            }
          }
          const uint64_t bin = __ballot(in);
          if (work) n_rel += __popcll(bin);
          // where the row stops, written by the lane that holds it (no cross-lane moves: masks only)
          const uint32_t sh = gi * SW;
          bool more;
          if (SPEC) {
            // the next chunk while this one is full and its last arc within budget; stopping, the
            // last lane records ptr = the chunk's end and nxt = its own latency (a lower bound of
            // the next arc's)
            const bool full = a[g] + SW < e[g];
            const uint64_t inb = __ballot(r[g].y <= budget[g]);
            more = full && (inb >> (sh + SW - 1) & 1u);
            if (!more && a[g] < e[g]) {
              if (full && gl == SW - 1) {
                ptr[u[g]] = a[g] + SW;
                nxt[u[g]] = r[g].y;
              } else if (!full && gl == 0) {
                ptr[u[g]] = e[g];
                nxt[u[g]] = LAT32_SAT;
              }
            }
          } else {
            // the group's first arc past the budget (its arcs are sorted: the in-lanes are a prefix)
            const uint64_t gmask = (SW == 64 ? ~0ull : ((1ull << SW) - 1ull)) << sh;
            const uint64_t stop = __ballot(i < e[g] && !in) & gmask;
            more = !stop && a[g] + SW < e[g];
            if (stop) {
              if (lane == (uint32_t)__builtin_ctzll(stop)) {
                ptr[u[g]] = i;
                nxt[u[g]] = r[g].y;
              }
            } else if (!more && a[g] < e[g] && gl == 0) {
              ptr[u[g]] = e[g];
              nxt[u[g]] = LAT32_SAT;
            }
          }
          a[g] = more ? a[g] + SW : e[g];
          more_any |= __ballot(more);
        }
        live = more_any != 0;
      }
    }
    for (int d = 32; d > 0; d >>= 1) mo = min(mo, (uint32_t)__shfl_xor(mo, d, 64));
    if (lane == 0 && mo < LAT32_SAT) atomicMin(&s_mo, mo);
    __syncthreads();
    DN_MARK(2);
    // 3. settle below min(thr, m2 + w_min); the next m (unsettled keys) and me (settled rows)
    const uint32_t m2 = s_mo;
    const uint32_t thr2 = min(thr, m2 + wmin >= m2 ? m2 + wmin : LAT32_SAT);
    uint32_t mn = LAT32_SAT, men = LAT32_SAT;
    for (uint32_t v = t; v < n; v += TH) {
      const uint32_t l = key_lat(key[v]);
      bool st = settled[v >> 5] >> (v & 31) & 1u;
      if (!st && l < thr2) {
        atomicOr(&settled[v >> 5], 1u << (v & 31));
        st = true;
        s_new = 1u;  // (benign race, as s_un)
      }
      if (st) men = min(men, __builtin_elementwise_add_sat(l, nxt[v]));
      else mn = min(mn, l);
      if (!st) s_un = 1u;  // (a benign race: every writer stores 1)
    }
    for (int d = 32; d > 0; d >>= 1) {
      mn = min(mn, (uint32_t)__shfl_xor(mn, d, 64));
      men = min(men, (uint32_t)__shfl_xor(men, d, 64));
    }
    if (lane == 0) {
      if (mn < LAT32_SAT) atomicMin(&s_m, mn);
      if (men < LAT32_SAT) atomicMin(&s_me, men);
    }
    if (t == 0) s_cnt = 0;
    __syncthreads();
    m = s_m;
    me = s_me;
    un = s_un;
    settled_any = s_new;
    __syncthreads();  // (s_m / s_me are reset by the next round's listing)
    DN_MARK(3);
  }
  if (work && lane == 0 && n_rel) atomicAdd(&work[blockIdx.x & 63], n_rel);
  dense_write_row<TH>(key, src, row, used, n_used, self_edge, e_lat, e_loss, out_lat + (size_t)blockIdx.x * n_used,
                      out_loss + (size_t)blockIdx.x * n_used, sat_row + blockIdx.x);
#ifdef DN_PROF
  DN_MARK(4);
  pt[7] = tq - t0q;
  if (t == 0)
    for (int k = 0; k < 8; k++) atomicAdd(&g_dn_prof[k], pt[k]);
#endif
#undef DN_MARK
}

bool sssp_dense_fits(uint32_t n) { return n > 0 && n <= DENSE_MAX; }

// rounds with fewer settled rows than this split each row over several waves (SG_DENSE_SPLIT;
// C2: 0.363 ms without, 0.320 below 4 rows, 0.305 below 8, 0.299 below 16, r8u)
static uint32_t dense_split_below(int waves) {
  const char* v = getenv("SG_DENSE_SPLIT");
  const int x = v && *v ? atoi(v) : waves;
  return (uint32_t)std::max(0, std::min(waves, x));
}

// threads per row (SG_DENSE_THREADS, SG_DENSE_SEED_THREADS for the seeded launches: 512 or 1024)
// and lanes per settled row in the relaxation (SG_DENSE_SW, SG_DENSE_SEED_SW: 8, 16, 32 or 64).
// C2 with 256 seed rows (r6, `profiles/r06/ab_c2_seed_r6.txt`): seeded 1024 threads x 64 lanes
// 0.261 ms, 512 x 64 0.243, 1024 x 16 0.222, 512 x 32 0.211, 512 x 16 0.195, 512 x 8 0.191; the
// unseeded launch at 32 lanes 0.198 against 0.196, at 16 lanes 0.218 (its early rounds read whole rows)
static int dense_env(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}

// rows of the launches before the last (SG_DENSE_SEED, a comma list, e.g. "32,224"; 0: one launch,
// no seeds; unset: one seed launch of n_cu rows); levels that would leave the last launch fewer
// rows than they hold are dropped.  C2 (r6, `profiles/r06/ab_c2_seed_r6.txt`): unseeded 0.297 ms;
// 128 / 256 / 384 / 512 seed rows 0.296 / 0.261 / 0.278 / 0.259; "32,224" 0.327, "16,112,384"
// 0.389 (every level costs one row's latency, ~75-85 us, whatever its size)
static std::vector<uint32_t> dense_seed_levels(uint32_t rows, uint32_t n_cu) {
  std::vector<uint32_t> lv;
  const char* v = getenv("SG_DENSE_SEED");
  if (!v || !*v) {
    if (rows >= 2 * n_cu) lv.push_back(n_cu);
    return lv;
  }
  uint64_t sum = 0;
  for (const char* p = v; *p;) {
    char* end;
    const long x = strtol(p, &end, 10);
    if (end == p) break;
    p = *end == ',' ? end + 1 : end;
    if (x <= 0 || rows < 2 * (sum + (uint64_t)x)) break;
    lv.push_back((uint32_t)x);
    sum += (uint64_t)x;
  }
  return lv;
}

void launch_sssp_dense(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used, uint32_t row_begin,
                       uint32_t row_end, uint64_t* out_lat, float* out_loss, uint32_t* sat_row,
                       unsigned long long* work) {
  const uint32_t n = net->n_nodes, rows = row_end - row_begin;
  if (!sssp_dense_fits(n)) throw Error(SG_ERR_INVALID_ARG, "graph too large for the dense search");
  if ((uint64_t)net->n_arcs * 4 * DN_W >= (1ull << 31)) throw Error(SG_ERR_INVALID_ARG, "too many arcs for the dense search");
  hipStream_t st = ctx->stream;
  // workspace: sorted arcs (4 DN_W B each), w_min, per-node sorted flag.  A graph is immutable,
  // so its arcs are sorted once: a rebuild on the same sg_net reuses them (the context's workspace
  // remembers whose arcs it holds; C2 rebuild 0.46 -> ~0.33 ms, the sort ~0.13 ms)
  const size_t words = (size_t)net->n_arcs * DN_W + 4 + (n + 3) / 4 + n;
  const bool fresh = ctx->dense_owner != net->serial || ctx->r_dense.cap < words * 4;
  uint32_t* sa = ctx->r_dense.get<uint32_t>(words);
  uint32_t* wmin = sa + (size_t)net->n_arcs * DN_W;
  uint8_t* sorted = (uint8_t*)(wmin + 4);
  uint32_t* mark = wmin + 4 + (n + 3) / 4;  // [n] seed-row stamps
  if (fresh) {
    ctx->dense_owner = 0;  // (set again once the sort is queued)
    TimedLaunch tl(ctx, "dense_sort", 24.0 * net->n_arcs);
    SG_HIP(hipMemsetAsync(wmin, 0xFF, 4, st));
    SG_HIP(hipMemsetAsync(mark, 0, (size_t)n * 4, st));
    ctx->dense_gen = 0;
    uint32_t cap = 64;
    while (cap < n - 1 && cap < SORT_MAXDEG) cap <<= 1;
    hipLaunchKernelGGL(k_sort_arcs, dim3(n), dim3(SORT_THREADS), cap * 8, st, net->out_off, net->out_arc, cap, sa,
                       sorted, wmin);
    SG_CHECK_LAUNCH();
    ctx->dense_owner = net->serial;
  }
  if (!rows) return;
  const uint32_t nbw = (n + 31) / 32;
  const size_t lds = (size_t)n * 8 + (size_t)((nbw + 1) & ~1u) * 4 + DENSE_SCAP * 4;
  auto launch = [&](uint32_t r0, uint32_t nr, DenseSeed sd) {
    // the arc record's size (bytes read per relaxation), for the roofline accounting of bench.py
    timer_add_work(ctx, "sssp_dense_rec_bytes", 4.0 * DN_W);
    TimedLaunch tl(ctx, "sssp_dense", 0.0);
    const size_t o = (size_t)(r0 - row_begin) * n_used;
    const bool seeded = sd.mode & DENSE_SEED_USE;
    const int th = dense_env(seeded ? "SG_DENSE_SEED_THREADS" : "SG_DENSE_THREADS", seeded ? 512 : DENSE_THREADS) == 512 ? 512 : 1024;
    const int sw = dense_env(seeded ? "SG_DENSE_SEED_SW" : "SG_DENSE_SW", seeded ? 8 : 64);
    auto pick = [](auto k8, auto k16, auto k32, auto k64, int w) { return w == 8 ? k8 : w == 16 ? k16 : w == 32 ? k32 : k64; };
    auto kern = th == 512 ? pick(k_sssp_dense<512, 8>, k_sssp_dense<512, 16>, k_sssp_dense<512, 32>, k_sssp_dense<512, 64>, sw)
                          : pick(k_sssp_dense<1024, 8>, k_sssp_dense<1024, 16>, k_sssp_dense<1024, 32>, k_sssp_dense<1024, 64>, sw);
    hipLaunchKernelGGL(kern, dim3(nr), dim3(th), lds, st, net->out_off, (const uint32_t*)sa,
                       (const uint8_t*)sorted, n, net->n_arcs, (const uint32_t*)wmin, d_used, n_used, r0,
                       net->self_edge, net->e_lat, net->e_loss, out_lat + o, out_loss + o, sat_row + (r0 - row_begin),
                       work, dense_split_below(th / 64), sd);
    SG_CHECK_LAUNCH();
  };
  // the lazy search (default; SG_DENSE_LAZY=0: the T-cut search with seed rows).  Latency-bound:
  // 64 rows take 75 us at 256 threads (50 at 512), all 1,200 92 us (106 at 512: past the 32
  // waves per CU); per row at 1,200 rows, 256 threads (a -DDN_PROF build): init 3.6 us, listing
  // 11.8, relaxation 61.1, settling 12.8, write-out 5.7 over 8 rounds and ~2,000 listed rows.  A
  // scheduling barrier that issues both rows' loads before the first use measured 0.127 ms against
  // 0.124 (not kept).  384 threads (6 waves; 1,200 rows still fit 32 waves per CU) 0.121-0.123
  // against 0.126-0.127 for 256 (rocprof 92 against ~97 us per rebuild launch), but its HIP-event
  // pair behind bench.py's spin kernel reads 0.118 ms, 26 us over the trace, so the line's
  // roofline would not match the profile: 256 stays the default.  The atomic's returned key
  // instead of a settled-bit read ahead of it (SG_DENSE_RTN, default) 0.125 against 0.126
  // (`profiles/r06/ab_c2_lazy_r6.txt`)  C2 (r6,
  // `profiles/r06/ab_c2_lazy_r6.txt`): T cut 0.297 ms, with 256 seed rows 0.190; lazy 512 threads x
  // 8 lanes 0.171, 256 x 4 0.151; lazy whole chunks (SG_DENSE_SPEC) 256 x 4 0.130, 256 x 8 0.124,
  // 256 x 16 0.126, 512 x 8 0.136; 4 rows in flight per lane group (SG_DENSE_G=4) 0.132-0.136
  if (dense_env("SG_DENSE_LAZY", 1)) {
    const int th0 = dense_env("SG_DENSE_THREADS", 256), th = th0 == 512 || th0 == 384 ? th0 : 256;
    const int sw = dense_env("SG_DENSE_SW", 8), gg = dense_env("SG_DENSE_G", 2) == 4 ? 4 : 2;
    const bool spec = dense_env("SG_DENSE_SPEC", 1) != 0;
#define SG_LAZY_K(T_, S_, G_) (spec ? k_sssp_dense_lazy<T_, S_, G_, true> : k_sssp_dense_lazy<T_, S_, G_, false>)
    auto pick = [&](auto k4, auto k8, auto k16) { return sw == 4 ? k4 : sw == 16 ? k16 : k8; };
    const bool rtn = dense_env("SG_DENSE_RTN", 1) != 0 && spec && sw == 8 && gg == 2;
    auto kern = rtn ? (th == 384 ? k_sssp_dense_lazy<384, 8, 2, true, true> : th == 512 ? k_sssp_dense_lazy<512, 8, 2, true, true>
                                                                               : k_sssp_dense_lazy<256, 8, 2, true, true>)
              : th == 256 ? (gg == 4 ? pick(SG_LAZY_K(256, 4, 4), SG_LAZY_K(256, 8, 4), SG_LAZY_K(256, 16, 4))
                                     : pick(SG_LAZY_K(256, 4, 2), SG_LAZY_K(256, 8, 2), SG_LAZY_K(256, 16, 2)))
              : th == 384 ? pick(SG_LAZY_K(384, 4, 2), SG_LAZY_K(384, 8, 2), SG_LAZY_K(384, 16, 2))
                          : (gg == 4 ? pick(SG_LAZY_K(512, 4, 4), SG_LAZY_K(512, 8, 4), SG_LAZY_K(512, 16, 4))
                                     : pick(SG_LAZY_K(512, 4, 2), SG_LAZY_K(512, 8, 2), SG_LAZY_K(512, 16, 2)));
#undef SG_LAZY_K
    const size_t lds_l = (size_t)n * 8 + (size_t)n * 16 + (size_t)nbw * 4;
    timer_add_work(ctx, "sssp_dense_rec_bytes", 4.0 * DN_W);
    TimedLaunch tl(ctx, "sssp_dense", 0.0);
    hipLaunchKernelGGL(kern, dim3(rows), dim3(th), lds_l, st, net->out_off, (const uint32_t*)sa, (const uint8_t*)sorted,
                       n, (const uint32_t*)wmin, d_used, n_used, row_begin, net->self_edge, net->e_lat, net->e_loss,
                       out_lat, out_loss, sat_row, work);
    SG_CHECK_LAUNCH();
#ifdef DN_PROF
    {
      unsigned long long h[8], z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      SG_HIP(hipStreamSynchronize(st));
      SG_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_dn_prof), sizeof(h)));
      SG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_dn_prof), z, sizeof(z)));
      const double r = rows ? (double)rows : 1.0;
      fprintf(stderr, "dense_prof rows %u per row (us): init %.2f list %.2f relax %.2f settle %.2f write %.2f "
              "whole %.2f rounds %.2f listed %.1f\n", rows, h[0] / r / 100, h[1] / r / 100, h[2] / r / 100,
              h[3] / r / 100, h[4] / r / 100, h[7] / r / 100 + h[0] / r / 100, h[5] / r, h[6] / r);
    }
#endif
    return;
  }
  const std::vector<uint32_t> lv = dense_seed_levels(rows, (uint32_t)std::max(1, ctx->n_cu));
  if (lv.empty()) {
    launch(row_begin, rows, DenseSeed{0, 0, 0, 0, nullptr, nullptr});
    return;
  }
  if (ctx->dense_gen + lv.size() + 1 > 0xFFFFu) {  // stamps would wrap: clear them
    SG_HIP(hipMemsetAsync(mark, 0, (size_t)n * 4, st));
    ctx->dense_gen = 0;
  }
  const uint32_t gen_lo = ctx->dense_gen + 1;  // this call's first stamp generation
  uint32_t r0 = row_begin;
  for (size_t l = 0; l <= lv.size(); l++) {
    const uint32_t nr = l < lv.size() ? lv[l] : row_end - r0;
    const uint32_t mode = (l < lv.size() ? DENSE_SEED_MARK : 0u) | (l ? DENSE_SEED_USE : 0u);
    launch(r0, nr, DenseSeed{mode, gen_lo, gen_lo + (uint32_t)l, row_begin, mark, out_lat});
    r0 += nr;
  }
  ctx->dense_gen = gen_lo + (uint32_t)lv.size();
}

}  // namespace sg
