// sg_dense.hip -- per-source shortest paths on dense graphs (C2: the 1,200-node
// complete graph of docs/network_graph_overview.md:58-63).
//
// Replaces, for graphs of at most DENSE_MAX nodes whose mean out-degree is past
// the sparse searches' range, the per-source petgraph::algo::dijkstra of
// NetworkGraph::compute_shortest_paths (graph/mod.rs:190-208).
//
// One workgroup per source row, its keys in LDS.  The search settles nodes in
// rounds (Dijkstra with a width) and relaxes only the arcs that can still matter:
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

#include "sg_device.h"
#include "sg_internal.h"

namespace sg {

#ifndef DN_THREADS  // (A/B builds: 512 and 256 threads per row measured 0.317-0.321 and 0.312-0.316 ms
#define DN_THREADS 1024  // against 0.301-0.303 at C2 with the row split, r8x)
#endif
constexpr int DENSE_THREADS = DN_THREADS;
constexpr int DENSE_WAVES = DENSE_THREADS / 64;
constexpr uint32_t DENSE_SCAP = 512;    // nodes settled per round at most (the rest wait a round)
constexpr uint32_t SORT_MAXDEG = 4096;  // out-degree sorted in one block's LDS; larger rows stay unsorted
#ifndef DN_G  // (A/B builds at C2, r8y: 1 row 0.320-0.323 ms, 3 rows 0.304-0.305, 4 rows 0.454-0.455, 2 rows 0.304-0.306)
#define DN_G 2
#endif
constexpr int DENSE_G = DN_G;           // settled rows a wave relaxes together (their loads in flight)
// Sorted-arc records of 12 B (b96 loads; DN_REC16 builds the 16-B records with a pad word of r04).
// A/B knobs (C2, r7h, `profiles/r05/ab_c2_dense_r7h.txt`): 12-B records 0.461-0.465 ms against
// 0.469-0.474 for 16 B; DN_NT1 (nt loads in a round whose cut is still open: a row's whole arc
// list, read once) 0.520; DN_NTOUT (nontemporal table stores) 0.470-0.472.
#ifndef DN_REC16
#define DN_REC12
#endif
#ifdef DN_REC12
constexpr uint32_t DN_W = 3;
#else
constexpr uint32_t DN_W = 4;
#endif

// Per node u: its out-arcs (out_arc, 3 u32 each: head, latency32, bits(1f32 - loss))
// sorted by latency into 16-B records {head, latency32, bits(om), 0} at the same
// offsets; sorted[u] = 1, or 0 for a row past `cap` arcs (copied as is, never cut
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

__global__ void __launch_bounds__(DENSE_THREADS) k_sssp_dense(const uint32_t* __restrict__ out_off,
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
                                                              uint32_t split_below) {
  extern __shared__ __align__(16) unsigned char smem[];
  unsigned long long* key = (unsigned long long*)smem;        // [n]
  uint32_t* settled = (uint32_t*)(key + n);                   // [ceil(n / 32)] bitmap
  const uint32_t nbw = (n + 31) / 32;
  uint32_t* s_node = settled + ((nbw + 1) & ~1u);             // [DENSE_SCAP] this round's settled nodes
  __shared__ uint32_t s_cnt;
  __shared__ uint32_t red_m[DENSE_WAVES], red_t[DENSE_WAVES];
  __shared__ uint32_t s_m, s_t;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t row = row_begin + blockIdx.x;
  const uint32_t src = used[row];
  const uint32_t wmin = *wmin_p;  // >= 1 (graph/mod.rs:105-107); LAT32_SAT: no arc at all
  for (uint32_t v = t; v < n; v += DENSE_THREADS) key[v] = v == src ? 0ull : KEY_INF;  // default() at the source
  for (uint32_t i = t; i < nbw; i += DENSE_THREADS) settled[i] = 0u;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)sa, 0, (int)0x7FFFFFFF, 0x00020000);
  unsigned long long n_rel = 0;
  __syncthreads();
  for (;;) {
    // the smallest and largest latency of the unsettled keys
    uint32_t m = LAT32_SAT, T = 0;
    for (uint32_t v = t; v < n; v += DENSE_THREADS) {
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
      for (int k = 0; k < DENSE_WAVES; k++) {
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
    for (uint32_t v0 = wv * 64; v0 < n; v0 += DENSE_THREADS) {
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
    // whole rows) splits each row over DENSE_WAVES / ns waves, which take its 64-arc chunks in
    // turn -- the row's loads in flight side by side instead of one chunk after the other.
    if (ns < split_below) {
      const uint32_t per = DENSE_WAVES / ns, r = wv % ns, p = wv / ns;
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
    for (uint32_t s0 = wv * DENSE_G; s0 < ns; s0 += DENSE_WAVES * DENSE_G) {
      uint32_t a[DENSE_G], e[DENSE_G];
      uint64_t ku[DENSE_G];
      bool cut[DENSE_G];
#pragma unroll
      for (int g = 0; g < DENSE_G; g++) {
        const bool ok = s0 + g < ns;
        const uint32_t u = ok ? s_node[s0 + g] : 0u;
        a[g] = ok ? out_off[u] : 0u;
        e[g] = ok ? out_off[u + 1] : 0u;
        ku[g] = ok ? key[u] : KEY_INF;
        cut[g] = ok && sorted[u];
      }
      // the latency budget of row g's arcs: key(u).lat + w <= T
      uint32_t budget[DENSE_G];
#pragma unroll
      for (int g = 0; g < DENSE_G; g++) budget[g] = T - min(T, key_lat(ku[g]));
      bool live = true;
#ifdef DN_NT1
      const bool open = T == LAT32_SAT;  // (uniform) an open cut: whole rows, read once
#endif
      while (live) {
        uint4 r[DENSE_G];
#pragma unroll
        for (int g = 0; g < DENSE_G; g++) {
          const uint32_t i = a[g] + lane;
          const uint32_t off = i < e[g] ? i * (4u * DN_W) : 0x80000000u;
#ifdef DN_REC12
#ifdef DN_NT1
          const auto x = open ? __builtin_amdgcn_raw_buffer_load_b96(ra, off, 0, 2)
                              : __builtin_amdgcn_raw_buffer_load_b96(ra, off, 0, 0);
#else
          const auto x = __builtin_amdgcn_raw_buffer_load_b96(ra, off, 0, 0);
#endif
          r[g] = make_uint4(x[0], x[1], x[2], 0u);
#else
#ifdef DN_NT1
          const auto x = open ? __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 2)
                              : __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0);
#else
          const auto x = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0);
#endif
          r[g] = make_uint4(x[0], x[1], x[2], x[3]);
#endif
        }
        live = false;
#pragma unroll
        for (int g = 0; g < DENSE_G; g++) {
          const uint32_t i = a[g] + lane;
          const bool in = i < e[g] && (!cut[g] || r[g].y <= budget[g]);
          const uint64_t cd = relax32(ku[g], r[g].y, __uint_as_float(r[g].z));
          const bool offer = in && key_lat(cd) != LAT32_SAT && !(settled[r[g].x >> 5] >> (r[g].x & 31) & 1u);
          if (offer) (void)__hip_atomic_fetch_min(&key[r[g].x], (unsigned long long)cd, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_WORKGROUP);
          if (work) n_rel += __popcll(__ballot(in));
          // the row goes on while its last lane's arc is in range and within the budget
          const bool more = __builtin_amdgcn_readlane((int)in, 63) != 0 && a[g] + 64 < e[g];
          a[g] = more ? a[g] + 64 : e[g];
          live |= more;
        }
      }
    }
    __syncthreads();
  }
  if (work && lane == 0 && n_rel) atomicAdd(&work[blockIdx.x & 63], n_rel);
  // ---- write the row: columns in used order, diagonal = the raw self-loop (graph/mod.rs:210-217)
  bool sat = false;
  const size_t orow = (size_t)blockIdx.x * n_used;
  const uint32_t de = self_edge[src];
  for (uint32_t jj = t; jj < n_used; jj += DENSE_THREADS) {
    const uint32_t v = used[jj];
    const unsigned long long k = key[v];
    const bool diag = jj == row;
    sat |= !diag && key_lat(k) == LAT32_SAT;
#ifdef DN_NTOUT
    __builtin_nontemporal_store(diag ? e_lat[de] : (uint64_t)key_lat(k), &out_lat[orow + jj]);
    __builtin_nontemporal_store(diag ? e_loss[de] : __uint_as_float(key_loss_bits(k)), &out_loss[orow + jj]);
#else
    out_lat[orow + jj] = diag ? e_lat[de] : (uint64_t)key_lat(k);
    out_loss[orow + jj] = diag ? e_loss[de] : __uint_as_float(key_loss_bits(k));
#endif
  }
  if (__any(sat) && lane == 0) sat_row[blockIdx.x] = 1u;
}

bool sssp_dense_fits(uint32_t n) { return n > 0 && n <= DENSE_MAX; }

// rounds with fewer settled rows than this split each row over several waves (SG_DENSE_SPLIT;
// C2: 0.363 ms without, 0.320 below 4 rows, 0.305 below 8, 0.299 below 16, r8u)
static uint32_t dense_split_below() {
  const char* v = getenv("SG_DENSE_SPLIT");
  const int x = v && *v ? atoi(v) : DENSE_WAVES;
  return (uint32_t)std::max(0, std::min(DENSE_WAVES, x));
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
  const size_t words = (size_t)net->n_arcs * DN_W + 4 + (n + 3) / 4;
  const bool fresh = ctx->dense_owner != net->serial || ctx->r_dense.cap < words * 4;
  uint32_t* sa = ctx->r_dense.get<uint32_t>(words);
  uint32_t* wmin = sa + (size_t)net->n_arcs * DN_W;
  uint8_t* sorted = (uint8_t*)(wmin + 4);
  if (fresh) {
    ctx->dense_owner = 0;  // (set again once the sort is queued)
    TimedLaunch tl(ctx, "dense_sort", 24.0 * net->n_arcs);
    SG_HIP(hipMemsetAsync(wmin, 0xFF, 4, st));
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
  // the arc record's size (bytes read per relaxation), for the roofline accounting of bench.py
  timer_add_work(ctx, "sssp_dense_rec_bytes", 4.0 * DN_W);
  TimedLaunch tl(ctx, "sssp_dense", 0.0);
  hipLaunchKernelGGL(k_sssp_dense, dim3(rows), dim3(DENSE_THREADS), lds, st, net->out_off, (const uint32_t*)sa,
                     (const uint8_t*)sorted, n, net->n_arcs, (const uint32_t*)wmin, d_used, n_used, row_begin,
                     net->self_edge, net->e_lat, net->e_loss, out_lat, out_loss, sat_row, work,
                     dense_split_below());
  SG_CHECK_LAUNCH();
}

}  // namespace sg
