// sg_routing.hip -- routing-table build on MI355X.
//
// Replaces NetworkGraph::compute_shortest_paths (graph/mod.rs:183-228) and
// NetworkGraph::get_direct_paths (graph/mod.rs:230-252).
//
// Shortest paths.  The reference runs petgraph's Dijkstra per used source
// over (latency u64, loss f32) with the LEFT fold default() + e1 + e2 + ...
// (graph/mod.rs:195-200, 322-331).  Because edge latency >= 1 ns
// (graph/mod.rs:105-107) and the f32 fold is monotone, that result equals the
// fixed point of the source-rooted relaxation
//     D[s][v] = min(D[s][v], D[s][u] (+) w(u,v))
// under ANY relaxation order, as long as every update keeps the edge on the
// right (source-rooted) and the (latency, loss) pair is updated atomically.
// Floyd-Warshall would re-associate the f32 fold and is not bit-exact for loss.
//
// Two kernels compute the same fixed point:
//  * sg_sssp.hip k_sssp_lds (graphs up to ~10.9k nodes, the default there): one
//    workgroup per source, the source's whole distance row in LDS, an
//    asynchronous work queue, rows bounded (and partly seeded exactly) by
//    neighbour rows finished in earlier phases; about 1.1-1.6x Dijkstra's
//    relaxations at C3.
//  * k_relax_w2 below (larger graphs): batched-source pull relaxation.  A wave
//    owns a few destination nodes of one 64-source batch; lane = source.  The
//    batch's distance slab is laid out [node][64 sources], so each in-arc
//    (u -> v) costs one coalesced 512-B read of D[u][0..63] and 64 independent
//    relaxations.
// Both use the packed key (latency u32 << 32) | f32 bits(loss) (sg_device.h), so
// one u64 min is the lexicographic PathProperties comparison.  Latency adds
// saturate at LAT32_SAT = 2^32 - 1 ns; rows holding a saturated key (a path of
// 4.29 s or more, or an unreachable node) are redone by the wide (u64 latency,
// f32 loss) Jacobi kernel k_relax_wide.
//
// In-place (Gauss-Seidel) updates in k_relax_w2.  A flush writes a lane's two
// keys with one 16-B store while other waves may gather the same row with 16-B
// loads.  Each key is one aligned 8-B half of that store.  MI355X_MICROARCH.md
// records untorn 16-B halves on gfx950 as observed, not architecturally
// guaranteed; the exactness argument needs only that each aligned 8-B key is
// read whole (a 64-bit access), which is how the vector memory path moves
// aligned dwordx2 halves.  Dense graphs (arc segments) flush with 64-bit
// atomicMin instead.  The LDS kernel updates keys with 64-bit LDS atomics.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <system_error>
#include <thread>
#include <type_traits>
#include <vector>

#include "sg_device.h"
#include "sg_internal.h"

namespace sg {

constexpr int BATCH = 64;         // sources per batch = wave width
constexpr int RELAX_WAVES = 4;    // waves per block (wide kernel)
constexpr int RELAX_BLOCK = RELAX_WAVES * 64;
constexpr int WORK_SHARDS = 64;  // relaxation counter shards (measurement only)

// ---------------------------------------------------------------------------
// Graph upload: CSC of in-arcs (both directions when undirected, petgraph
// semantics graph/mod.rs:137-152), self-loop census for get_edge_weight(n, n).
// ---------------------------------------------------------------------------
// The upload's two zero fills (the degree counters, the self-loop census) as one launch:
// two hipMemsetAsync calls cost ~16 us of host time and two fill dispatches on the device
__global__ void k_zero2(uint32_t* __restrict__ a, uint32_t na, uint32_t* __restrict__ b, uint32_t nb) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < na + nb; i += gridDim.x * blockDim.x) {
    if (i < na) a[i] = 0u;
    else b[i - na] = 0u;
  }
}

// One pass over the edges for both arc lists and the self-loop census (a graph
// upload is part of every one-shot build: three launches instead of six).
__global__ void k_net_count(const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst, uint32_t m,
                            int directed, uint32_t* __restrict__ indeg, uint32_t* __restrict__ outdeg,
                            uint32_t* __restrict__ self_cnt, uint32_t* __restrict__ self_edge) {
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < m; e += gridDim.x * blockDim.x) {
    const uint32_t s = src[e], d = dst[e];
    if (s == d) {
      atomicAdd(&self_cnt[s], 1u);
      self_edge[s] = e;  // meaningful only when the count ends at 1
      continue;
    }
    atomicAdd(&indeg[d], 1u);
    atomicAdd(&outdeg[s], 1u);
    if (!directed) {
      atomicAdd(&indeg[s], 1u);
      atomicAdd(&outdeg[d], 1u);
    }
  }
}

// Graphs of up to NET_LDS_NODES nodes (C2: a 1,200-node complete graph, 720k edges)
// count and place their arcs through per-block LDS counters: the global degree and
// cursor atomics of k_net_count / k_net_scatter all land on a few thousand words there
// (C2: 0.63 + 1.39 ms).  A block takes a contiguous run of edges; it adds its per-node
// counts to the global ones once, and reserves each node's range for its arcs with one
// returning atomic per node, then places them with LDS cursors.
constexpr uint32_t NET_LDS_NODES = 4096;
constexpr uint32_t NET_LDS_BLOCKS = 256;
__global__ void __launch_bounds__(256) k_net_count_lds(const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                                                       uint32_t m, uint32_t n, int directed,
                                                       uint32_t* __restrict__ indeg, uint32_t* __restrict__ outdeg,
                                                       uint32_t* __restrict__ self_cnt,
                                                       uint32_t* __restrict__ self_edge) {
  __shared__ uint32_t s_in[NET_LDS_NODES], s_out[NET_LDS_NODES];
  for (uint32_t v = threadIdx.x; v < n; v += 256) s_in[v] = s_out[v] = 0;
  __syncthreads();
  const uint32_t per = (m + gridDim.x - 1) / gridDim.x, e0 = blockIdx.x * per, e1 = min(e0 + per, m);
  for (uint32_t e = e0 + threadIdx.x; e < e1; e += 256) {
    const uint32_t s = src[e], d = dst[e];
    if (s == d) {
      atomicAdd(&self_cnt[s], 1u);
      self_edge[s] = e;  // meaningful only when the count ends at 1
      continue;
    }
    atomicAdd(&s_in[d], 1u);
    atomicAdd(&s_out[s], 1u);
    if (!directed) {
      atomicAdd(&s_in[s], 1u);
      atomicAdd(&s_out[d], 1u);
    }
  }
  __syncthreads();
  for (uint32_t v = threadIdx.x; v < n; v += 256) {
    if (s_in[v]) atomicAdd(&indeg[v], s_in[v]);
    if (s_out[v]) atomicAdd(&outdeg[v], s_out[v]);
  }
}

// OUT: the out-arcs (out_arc, every search's input) -- the upload; CSC: the in-arcs (in_src,
// in_lat, in_om, in_rec: the slab and wide kernels' and a directed plan's input) -- built on
// first use (ensure_csc), so an upload writes 12 B per arc instead of 52.
template <bool OUT, bool CSC>
__global__ void __launch_bounds__(256) k_net_scatter_lds(const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                                                         const uint64_t* __restrict__ lat, const float* __restrict__ loss,
                                                         uint32_t m, uint32_t n, int directed,
                                                         uint32_t* __restrict__ cursor, uint32_t* __restrict__ in_src,
                                                         uint64_t* __restrict__ in_lat, float* __restrict__ in_om,
                                                         uint4* __restrict__ in_rec, uint32_t* __restrict__ ocursor,
                                                         uint32_t* __restrict__ out_arc) {
  __shared__ uint32_t s_in[NET_LDS_NODES], s_out[NET_LDS_NODES];  // counts, then the block's cursors
  for (uint32_t v = threadIdx.x; v < n; v += 256) s_in[v] = s_out[v] = 0;
  __syncthreads();
  const uint32_t per = (m + gridDim.x - 1) / gridDim.x, e0 = blockIdx.x * per, e1 = min(e0 + per, m);
  for (uint32_t e = e0 + threadIdx.x; e < e1; e += 256) {
    const uint32_t s = src[e], d = dst[e];
    if (s == d) continue;
    if (CSC) atomicAdd(&s_in[d], 1u);
    if (OUT) atomicAdd(&s_out[s], 1u);
    if (!directed) {
      if (CSC) atomicAdd(&s_in[s], 1u);
      if (OUT) atomicAdd(&s_out[d], 1u);
    }
  }
  __syncthreads();
  for (uint32_t v = threadIdx.x; v < n; v += 256) {  // this block's ranges
    if (CSC && s_in[v]) s_in[v] = atomicAdd(&cursor[v], s_in[v]);
    if (OUT && s_out[v]) s_out[v] = atomicAdd(&ocursor[v], s_out[v]);
  }
  __syncthreads();
  for (uint32_t e = e0 + threadIdx.x; e < e1; e += 256) {
    const uint32_t s = src[e], d = dst[e];
    if (s == d) continue;  // a self-loop never improves D[s][v] (latency >= 1)
    const float om = __fsub_rn(1.0f, loss[e]);
    const uint64_t l = lat[e];
    const uint32_t l32 = l < LAT32_SAT ? (uint32_t)l : LAT32_SAT;
    for (int dir = 0; dir < (directed ? 1 : 2); dir++) {
      const uint32_t a = dir ? d : s, b = dir ? s : d;  // the arc a -> b
      if (CSC) {
        const uint32_t p = atomicAdd(&s_in[b], 1u);
        in_src[p] = a;
        in_lat[p] = l;
        in_om[p] = om;
        in_rec[p] = make_uint4(a, b, l32, __float_as_uint(om));
      }
      if (OUT) {
        const uint32_t q = atomicAdd(&s_out[a], 1u);
        out_arc[3 * (size_t)q] = b;
        out_arc[3 * (size_t)q + 1] = l32;
        out_arc[3 * (size_t)q + 2] = __float_as_uint(om);
      }
    }
  }
}

// Exclusive scans of indeg and outdeg (n + 1 entries each, the last one the
// total) in one workgroup, each result written twice: the offsets and the
// scatter's cursors.  For graphs up to NET_SCAN_SMALL nodes.  Both arrays in one
// pass over chunks of 16 x 1024 consecutive entries (32 branch-free loads in flight
// per thread); a thread's running offset carries across chunks in a register, and
// the offsets go out through LDS as coalesced stores.  (The earlier form gave each
// thread 10+ strided entries, one array at a time: 22 us at C3; with 8 entries per
// thread and stores straight from registers, 28 us; through LDS, 14.7 us.)
constexpr uint32_t NET_SCAN_SMALL = 1u << 17;
__global__ void __launch_bounds__(1024) k_net_scan(const uint32_t* __restrict__ indeg, const uint32_t* __restrict__ outdeg,
                                                   uint32_t n, uint32_t* __restrict__ in_off, uint32_t* __restrict__ in_cur,
                                                   uint32_t* __restrict__ out_off, uint32_t* __restrict__ out_cur) {
  constexpr int PER = 16;  // one chunk up to 16,383 nodes
  __shared__ uint32_t s_w[2][16];
  __shared__ uint32_t s_x[2][PER * 1024];  // 128 KB
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // branch-free loads (past n: an out-of-range offset reads 0), so all 16 are in flight
  // at once; with a branch per element the compiler waited for each load in turn
  const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void*)indeg, 0, (int)(n * 4u), 0x00020000);
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)outdeg, 0, (int)(n * 4u), 0x00020000);
  uint32_t carry_i = 0, carry_o = 0;
  for (uint32_t base = 0; base <= n; base += PER * 1024) {
    uint32_t xi[PER], xo[PER];
    uint32_t si = 0, so = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const uint32_t i = base + (uint32_t)tid * PER + k;
      xi[k] = __builtin_amdgcn_raw_buffer_load_b32(ri, i < n ? i * 4u : 0x80000000u, 0, 0);
      xo[k] = __builtin_amdgcn_raw_buffer_load_b32(ro, i < n ? i * 4u : 0x80000000u, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < PER; k++) {
      si += xi[k];
      so += xo[k];
    }
    const uint32_t ii = wave_incl_sum(si), io = wave_incl_sum(so);
    if (lane == 63) {
      s_w[0][wv] = ii;
      s_w[1][wv] = io;
    }
    __syncthreads();
    uint32_t pi = carry_i + ii - si, po = carry_o + io - so;
    for (int w = 0; w < 16; w++) {
      const uint32_t a = s_w[0][w], b = s_w[1][w];
      pi += w < wv ? a : 0u;
      po += w < wv ? b : 0u;
      carry_i += a;
      carry_o += b;
    }
    // the chunk's offsets through LDS, then stored coalesced (entry base + k * 1024 + tid)
#pragma unroll
    for (int k = 0; k < PER; k++) {
      s_x[0][tid * PER + k] = pi;
      s_x[1][tid * PER + k] = po;
      pi += xi[k];
      po += xo[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const uint32_t i = base + (uint32_t)k * 1024 + tid;
      const uint32_t a = s_x[0][k * 1024 + tid], b = s_x[1][k * 1024 + tid];
      if (i <= n) {
        in_off[i] = a;
        in_cur[i] = a;
        out_off[i] = b;
        out_cur[i] = b;
      }
    }
    __syncthreads();  // s_w and s_x are rewritten by the next chunk
  }
}

template <bool OUT, bool CSC>  // (as k_net_scatter_lds)
__global__ void k_net_scatter(const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                              const uint64_t* __restrict__ lat, const float* __restrict__ loss, uint32_t m,
                              int directed, uint32_t* __restrict__ cursor, uint32_t* __restrict__ in_src,
                              uint64_t* __restrict__ in_lat, float* __restrict__ in_om, uint4* __restrict__ in_rec,
                              uint32_t* __restrict__ ocursor, uint32_t* __restrict__ out_arc) {
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < m; e += gridDim.x * blockDim.x) {
    const uint32_t s = src[e], d = dst[e];
    if (s == d) continue;  // a self-loop never improves D[s][v] (latency >= 1)
    const float om = __fsub_rn(1.0f, loss[e]);
    const uint64_t l = lat[e];
    const uint32_t l32 = l < LAT32_SAT ? (uint32_t)l : LAT32_SAT;
    for (int dir = 0; dir < (directed ? 1 : 2); dir++) {
      const uint32_t a = dir ? d : s, b = dir ? s : d;  // the arc a -> b
      if (CSC) {
        const uint32_t p = atomicAdd(&cursor[b], 1u);
        in_src[p] = a;
        in_lat[p] = l;
        in_om[p] = om;
        in_rec[p] = make_uint4(a, b, l32, __float_as_uint(om));
      }
      if (OUT) {
        const uint32_t q = atomicAdd(&ocursor[a], 1u);
        out_arc[3 * (size_t)q] = b;
        out_arc[3 * (size_t)q + 1] = l32;
        out_arc[3 * (size_t)q + 2] = __float_as_uint(om);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Batched-source relaxation (the hot kernel).
//
// B sources per batch (lane = source).  A batch's distance slab is laid out
// D[node][B] (u64 keys, 8 B x B per node), so one in-arc u -> v costs one
// coalesced row read of D[u][0..B-1] and B independent relaxations.
//
// k_relax_w: one wave per work item (active batch, NPW consecutive destination
// nodes); see the kernel's comment.  XCD-aware 1-D grid: dispatch deals blocks
// round-robin over the 8 XCDs (MI355X_MICROARCH.md, "Workgroup dispatch"), so
// block L runs on XCD L % 8, and the items of one batch all go to blocks of one
// residue: the waves of an XCD share a slab in its L2.  Placement changes speed
// only, never results.
//
// Frontier (FRONT): stamp[batch][node] = p + 2 when the node's key changed in
// pass p (sources start at 1).  In pass p an arc is relaxed only when its
// source's stamp >= p + 1, i.e. the source changed in pass p - 1 or earlier in
// pass p.  Exactness: a value written in pass p is re-read by every out-arc in
// pass p + 1 (a kernel boundary, so visible), and iteration stops only after a
// pass with no change anywhere -- then every arc satisfies D[v] <= D[u] (+) w,
// the fixed point, which is petgraph's Dijkstra result (see header).
// ---------------------------------------------------------------------------
constexpr int RELAX_THREADS = 256;
constexpr uint32_t FLAG_STRIDE = 32;  // per-batch pass flags 128 B apart: no two batches share a cache line

// One 8-B key through a buffer descriptor (32-bit per-lane byte offset).  An
// offset of OOB lies outside every slab: the load returns 0 and moves no data.
constexpr uint32_t OOB = 0x80000000u;
constexpr uint32_t PREFETCH_MIN = 16;  // dirty arcs from which an item prefetches all its rows
__device__ __forceinline__ uint64_t load_key(__amdgpu_buffer_rsrc_t rsrc, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, off, 0, 0);
  return ((uint64_t)v[1] << 32) | v[0];
}

// Slab init: every key KEY_INF (16-B stores, no per-element index arithmetic),
// every stamp 0; k_stamp_sources then marks the sources.  (An earlier version
// tested each element against its batch's sources with 64-bit divisions and
// ran at about 0.3 TB/s.)
template <int B>
__global__ void k_init_batch(uint64_t* __restrict__ D, uint32_t* __restrict__ stamp, uint32_t n,
                             uint32_t n_batches) {
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  const size_t pairs = (size_t)n_batches * n * (B / 2), stride = (size_t)gridDim.x * blockDim.x;
  const u64x2 inf = {KEY_INF, KEY_INF};
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < pairs; i += stride)
    __builtin_nontemporal_store(inf, (u64x2*)D + i);
  const size_t ns = (size_t)n_batches * n;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += stride) stamp[i] = 0;
}

// Sources: key 0 (PathProperties::default()) and stamp 1, one thread per row.
template <int B>
__global__ void k_stamp_sources(uint64_t* __restrict__ D, uint32_t* __restrict__ stamp, uint32_t n,
                                const uint32_t* __restrict__ used, uint32_t first_row, uint32_t row_end,
                                uint32_t n_batches) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_batches * B) return;
  const uint32_t row = first_row + t;
  if (row >= row_end) return;
  const size_t bv = (size_t)(t / B) * n + used[row];
  stamp[bv] = 1;
  D[bv * B + (t % B)] = 0ull;
}

// Active-batch list for the next pass: alist[0] = count, alist[1 + i] = the
// i-th batch (ascending) whose flag is set.  One block.  Also zeroes the flag
// slot the pass will set (`clear`, gb x FLAG_STRIDE words) and, if count_out
// (pinned host-mapped) is given, reports the count there: no fill and no copy
// per pass.
__global__ void __launch_bounds__(1024) k_active_list(const uint32_t* __restrict__ flags, uint32_t gb,
                                                      uint32_t* __restrict__ alist, uint32_t* __restrict__ clear,
                                                      uint32_t* __restrict__ count_out) {
  for (uint32_t i = threadIdx.x; i < gb * FLAG_STRIDE; i += 1024) clear[i] = 0;
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t base;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint32_t b0 = 0; b0 < gb; b0 += 1024) {
    const uint32_t b = b0 + threadIdx.x;
    const bool on = b < gb && flags[b * FLAG_STRIDE] != 0;
    const uint64_t m = __ballot(on);
    if (lane == 0) wsum[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = base;
    for (int i = 0; i < wv; i++) off += wsum[i];
    if (on) alist[1 + off + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = b;
    __syncthreads();
    if (threadIdx.x == 0)
      for (int i = 0; i < 16; i++) base += wsum[i];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    alist[0] = base;
    if (count_out) *count_out = base;
  }
}

// B = sources per batch (64: one row per wave instruction; 32: two rows, one
// per half-wave, and a 2.5 MB slab at 10k nodes that stays in one XCD's L2).
template <int B, int NPW, int K, int GROUP, bool FRONT, bool COUNT>
__global__ void __launch_bounds__(RELAX_THREADS)
    k_relax_w(const uint32_t* __restrict__ in_off, const uint4* __restrict__ in_rec, uint64_t* __restrict__ D,
              uint32_t n, const uint32_t* __restrict__ alist, uint32_t* __restrict__ changed,
              uint32_t* __restrict__ stamp, uint32_t pass, unsigned long long* __restrict__ work) {
  constexpr int WAVES = RELAX_THREADS / 64;
  constexpr int STG_W = 64 * K;
  constexpr int G = 64 / B;  // rows per wave instruction
  static_assert(NPW % G == 0, "NPW must be a multiple of the rows per instruction");
  __shared__ uint4 lists[WAVES][STG_W];  // (source row byte offset, destination slot, latency, 1 - loss)
  __shared__ unsigned long long bests[WAVES][NPW * B];
  const int lane = threadIdx.x & 63;
  const uint32_t gh = lane / B, sl = lane % B;  // row group within the instruction, source lane
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane8 = sl * 8;
  uint4* list = lists[w];
  unsigned long long* best = bests[w];
  // Work items (active batch, wave chunk): the active batches with list index
  // i = x (mod 8) go to the blocks L = x (mod 8), i.e. to XCD x under
  // round-robin dispatch, so the remaining work stays spread over all XCDs as
  // batches converge; consecutive items are consecutive chunks of one batch, so
  // an XCD's resident waves share a slab.
  const uint32_t x = blockIdx.x & 7;
  const uint32_t nwc = (n + NPW - 1) / NPW;
  const uint32_t n_act = alist[0];
  const uint32_t nbx = n_act > x ? (n_act - x + 7) / 8 : 0;
  constexpr uint32_t nseg = 1;  // (segments: k_relax_w2 only)
  // nseg > 1 (dense graphs): an item is one of nseg segments of a node chunk's
  // in-arcs, so a chunk's thousands of arcs are relaxed by nseg waves at once;
  // the segments' waves share rows and merge by 64-bit atomic min (the packed
  // key's order is the PathProperties order)
  const uint32_t items = nbx * nwc * nseg;
  const uint32_t stride = (gridDim.x >> 3) * WAVES;
  uint32_t n_rel = 0, flagged = ~0u;
  for (uint32_t it = (blockIdx.x >> 3) * WAVES + w; it < items; it += stride) {
    const uint32_t b = alist[1 + x + 8 * (it / (nwc * nseg))];
    const uint32_t ci = it % (nwc * nseg);
    const uint32_t vw = (ci / nseg) * NPW, seg = ci % nseg;
    const uint32_t vw1 = min(vw + NPW, n);
    uint64_t* Db = D + (size_t)b * n * B;
    const uint32_t* St = stamp + (size_t)b * n;
    const __amdgpu_buffer_rsrc_t slab = __builtin_amdgcn_make_buffer_rsrc(Db, 0, (int)(n * B * 8u), 0x00020000);
    uint32_t a0 = in_off[vw], a1 = in_off[vw1];
    if (nseg > 1) {
      const uint32_t per = (a1 - a0 + nseg - 1) / nseg;
      a0 = min(a1, a0 + seg * per);
      a1 = min(a1, a0 + per);
    }
    uint32_t n_cand = 0;
    uint32_t run_slot = 0;  // per row group: records of one destination form a run
    uint64_t run = KEY_INF;
    bool prefetched = false;
    uint64_t cur[NPW / G];
    for (uint32_t c0 = a0; c0 < a1; c0 += STG_W) {
      const uint32_t c1 = min(c0 + STG_W, a1);
      uint4 ra[K];
      bool dirty[K];
#pragma unroll
      for (int i = 0; i < K; i++) ra[i] = in_rec[min(c0 + lane + 64 * i, c1 - 1)];
#pragma unroll
      for (int i = 0; i < K; i++) dirty[i] = c0 + lane + 64 * i < c1 && (!FRONT || St[ra[i].x] > pass);
      uint32_t cnt = 0;
#pragma unroll
      for (int i = 0; i < K; i++) {
        const uint64_t m = __ballot(dirty[i]);
        if (dirty[i])
          list[cnt + (uint32_t)__popcll(m & ((1ull << lane) - 1))] =
              make_uint4(ra[i].x * (B * 8), ra[i].y - vw, ra[i].z, ra[i].w);
        cnt += (uint32_t)__popcll(m);
      }
      if (cnt && !n_cand) {  // first candidates of this item: reset its LDS rows
#pragma unroll
        for (int i = 0; i < NPW * B / 64; i++) best[i * 64 + lane] = KEY_INF;
      }
      n_cand += cnt;
      if (cnt >= PREFETCH_MIN && !prefetched) {  // dense item: fetch its rows now, under the relax loop
        prefetched = true;
#pragma unroll
        for (int i = 0; i < NPW / G; i++)
          cur[i] = load_key(slab, min(vw + i * G + gh, vw1 - 1) * (B * 8) + lane8);
      }
      // Records arrive in destination order (CSC order, compaction keeps it);
      // row group gh takes records gh, gh + G, ..., so each destination's
      // candidates form one run per group, folded in registers and merged into
      // the destination's LDS row (ds_min) when the destination changes.
      uint32_t g = 0;
      for (; g + GROUP * G <= cnt; g += GROUP * G) {
        uint4 r[GROUP];
        uint64_t k[GROUP];
#pragma unroll
        for (int j = 0; j < GROUP; j++) r[j] = list[g + j * G + gh];
#pragma unroll
        for (int j = 0; j < GROUP; j++) k[j] = load_key(slab, r[j].x + lane8);
#pragma unroll
        for (int j = 0; j < GROUP; j++) {
          const uint32_t slot = G == 1 ? __builtin_amdgcn_readfirstlane(r[j].y) : r[j].y;
          if (slot != run_slot) {
            atomicMin(&best[run_slot * B + sl], (unsigned long long)run);
            run_slot = slot;
            run = KEY_INF;
          }
          run = min(run, relax32(k[j], r[j].z, __uint_as_float(r[j].w)));
        }
      }
      for (; g < cnt; g += G) {
        const uint32_t idx = g + gh;
        if (idx < cnt) {
          const uint4 r = list[idx];
          if (r.y != run_slot) {
            atomicMin(&best[run_slot * B + sl], (unsigned long long)run);
            run_slot = r.y;
            run = KEY_INF;
          }
          run = min(run, relax32(load_key(slab, r.x + lane8), r.z, __uint_as_float(r.w)));
        }
      }
    }
    if (COUNT) n_rel += n_cand;
    if (!n_cand) continue;
    atomicMin(&best[run_slot * B + sl], (unsigned long long)run);
    // flush: improved keys are written in place (one untorn 64-bit update each).
    // A sparse item reads only the lanes that received a candidate (the others
    // take an out-of-range offset: no memory traffic, value 0, no change).
    uint64_t nbv[NPW / G];
#pragma unroll
    for (int i = 0; i < NPW / G; i++) nbv[i] = best[(i * G + gh) * B + sl];
    if (!prefetched) {
#pragma unroll
      for (int i = 0; i < NPW / G; i++)
        cur[i] = load_key(slab, nbv[i] != KEY_INF ? min(vw + i * G + gh, vw1 - 1) * (B * 8) + lane8 : OOB);
    }
    bool any = false;
#pragma unroll
    for (int i = 0; i < NPW / G; i++) {
      const uint32_t v = vw + i * G + gh;
      const uint64_t nb = nbv[i];
      const bool ch = v < vw1 && nb < cur[i];
      if (ch) Db[(size_t)v * B + sl] = nb;
      const uint64_t m = __ballot(ch);
      if (m) {
        any = true;
        if (FRONT && sl == 0 && ((m >> (gh * B)) & (B == 64 ? ~0ull : ((1ull << B) - 1))))
          stamp[(size_t)b * n + v] = pass + 2;
      }
    }
    // one flag store per wave and batch (a wave's items run batch by batch)
    if (any && b != flagged) {
      if (lane == 0) changed[b * FLAG_STRIDE] = 1u;
      flagged = b;
    }
  }
  if (COUNT && lane == 0 && n_rel) atomicAdd(&work[blockIdx.x & (WORK_SHARDS - 1)], (unsigned long long)n_rel * B);
}

// Two 8-B keys (16 B) through the buffer descriptor; OOB -> zeros, no traffic.
__device__ __forceinline__ void load_key2(__amdgpu_buffer_rsrc_t rsrc, uint32_t off, uint64_t& k0, uint64_t& k1) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
  k0 = ((uint64_t)v[1] << 32) | v[0];
  k1 = ((uint64_t)v[3] << 32) | v[2];
}

// k_relax_w2: the B = 64 relaxation with two sources per lane.  A row (64 keys,
// 512 B) is read by 32 lanes with 16-B loads, so one wave instruction reads
// two rows (two arcs, one per half-wave): half the vector-memory instructions
// per relaxation.  The texture-address unit, 80 % busy in k_relax_w (PMC
// TA_TA_BUSY), processes one instruction's 64 addresses whatever their width.
// Same work items, frontier, LDS merge and flush as k_relax_w; a flush writes
// both keys of a lane with one 16-B store (the row's only writer is this wave,
// so the unchanged half is rewritten with the value it holds).
// B = 32 (SG_APSP_B=32): 16 lanes per row, four rows per wave instruction, and
// a 2.5 MB slab at 10k nodes that fits one XCD's 4 MB L2.
template <int B, int NPW, int K, int GROUP, bool FRONT, bool COUNT>
__global__ void __launch_bounds__(RELAX_THREADS)
    k_relax_w2(const uint32_t* __restrict__ in_off, const uint4* __restrict__ in_rec, uint64_t* __restrict__ D,
               uint32_t n, const uint32_t* __restrict__ alist, uint32_t* __restrict__ changed,
               uint32_t* __restrict__ stamp, uint32_t pass, unsigned long long* __restrict__ work, uint32_t nseg) {
  static_assert(B == 64 || B == 32, "B = 64 or 32");
  constexpr int WAVES = RELAX_THREADS / 64;
  constexpr int STG_W = 64 * K;
  constexpr int LPR = B / 2;   // lanes per row
  constexpr int G = 64 / LPR;  // rows per wave instruction
  constexpr uint64_t ROW_MASK = LPR == 64 ? ~0ull : (1ull << LPR) - 1;
  static_assert(NPW % G == 0, "NPW must be a multiple of the rows per instruction");
  __shared__ uint4 lists[WAVES][STG_W];
  __shared__ unsigned long long bests[WAVES][NPW * B];
  const int lane = threadIdx.x & 63;
  const uint32_t gh = lane / LPR, sl = lane % LPR;  // row group; the lane's sources 2 sl, 2 sl + 1
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane16 = sl * 16;
  uint4* list = lists[w];
  unsigned long long* best = bests[w];
  const uint32_t x = blockIdx.x & 7;
  const uint32_t nwc = (n + NPW - 1) / NPW;
  const uint32_t n_act = alist[0];
  const uint32_t nbx = n_act > x ? (n_act - x + 7) / 8 : 0;
  // nseg > 1 (dense graphs): an item is one of nseg segments of a node chunk's
  // in-arcs, so a chunk's thousands of arcs are relaxed by nseg waves at once;
  // the segments' waves share rows and merge by 64-bit atomic min (the packed
  // key's order is the PathProperties order)
  const uint32_t items = nbx * nwc * nseg;
  const uint32_t stride = (gridDim.x >> 3) * WAVES;
  uint32_t n_rel = 0, flagged = ~0u;
  for (uint32_t it = (blockIdx.x >> 3) * WAVES + w; it < items; it += stride) {
    const uint32_t b = alist[1 + x + 8 * (it / (nwc * nseg))];
    const uint32_t ci = it % (nwc * nseg);
    const uint32_t vw = (ci / nseg) * NPW, seg = ci % nseg;
    const uint32_t vw1 = min(vw + NPW, n);
    uint64_t* Db = D + (size_t)b * n * B;
    const uint32_t* St = stamp + (size_t)b * n;
    const __amdgpu_buffer_rsrc_t slab = __builtin_amdgcn_make_buffer_rsrc(Db, 0, (int)(n * B * 8u), 0x00020000);
    uint32_t a0 = in_off[vw], a1 = in_off[vw1];
    if (nseg > 1) {
      const uint32_t per = (a1 - a0 + nseg - 1) / nseg;
      a0 = min(a1, a0 + seg * per);
      a1 = min(a1, a0 + per);
    }
    uint32_t n_cand = 0;
    uint32_t run_slot = 0;
    uint64_t run0 = KEY_INF, run1 = KEY_INF;
    bool prefetched = false;
    uint64_t cur0[NPW / G], cur1[NPW / G];
    for (uint32_t c0 = a0; c0 < a1; c0 += STG_W) {
      const uint32_t c1 = min(c0 + STG_W, a1);
      uint4 ra[K];
      bool dirty[K];
#pragma unroll
      for (int i = 0; i < K; i++) ra[i] = in_rec[min(c0 + lane + 64 * i, c1 - 1)];
#pragma unroll
      for (int i = 0; i < K; i++) dirty[i] = c0 + lane + 64 * i < c1 && (!FRONT || St[ra[i].x] > pass);
      uint32_t cnt = 0;
#pragma unroll
      for (int i = 0; i < K; i++) {
        const uint64_t m = __ballot(dirty[i]);
        if (dirty[i])
          list[cnt + (uint32_t)__popcll(m & ((1ull << lane) - 1))] =
              make_uint4(ra[i].x * (B * 8), ra[i].y - vw, ra[i].z, ra[i].w);
        cnt += (uint32_t)__popcll(m);
      }
      if (cnt && !n_cand) {
#pragma unroll
        for (int i = 0; i < NPW * B / 64; i++) best[i * 64 + lane] = KEY_INF;
      }
      n_cand += cnt;
      if (cnt >= PREFETCH_MIN && !prefetched) {
        prefetched = true;
#pragma unroll
        for (int i = 0; i < NPW / G; i++)
          load_key2(slab, min(vw + i * G + gh, vw1 - 1) * (B * 8) + lane16, cur0[i], cur1[i]);
      }
      // half-wave gh takes records gh, gh + 2, ...: each destination's candidates
      // form one run per half-wave (CSC order)
      auto fold = [&](const uint4& r, uint64_t k0, uint64_t k1) {
        if (r.y != run_slot) {
          atomicMin(&best[run_slot * B + 2 * sl], (unsigned long long)run0);
          atomicMin(&best[run_slot * B + 2 * sl + 1], (unsigned long long)run1);
          run_slot = r.y;
          run0 = run1 = KEY_INF;
        }
        const float om = __uint_as_float(r.w);
        run0 = min(run0, relax32(k0, r.z, om));
        run1 = min(run1, relax32(k1, r.z, om));
      };
      uint32_t g = 0;
      for (; g + GROUP * G <= cnt; g += GROUP * G) {
        uint4 r[GROUP];
        uint64_t k0[GROUP], k1[GROUP];
#pragma unroll
        for (int j = 0; j < GROUP; j++) r[j] = list[g + j * G + gh];
#pragma unroll
        for (int j = 0; j < GROUP; j++) load_key2(slab, r[j].x + lane16, k0[j], k1[j]);
#pragma unroll
        for (int j = 0; j < GROUP; j++) fold(r[j], k0[j], k1[j]);
      }
      for (; g < cnt; g += G) {
        const uint32_t idx = g + gh;
        if (idx < cnt) {
          const uint4 r = list[idx];
          uint64_t k0, k1;
          load_key2(slab, r.x + lane16, k0, k1);
          fold(r, k0, k1);
        }
      }
    }
    if (COUNT) n_rel += n_cand;
    if (!n_cand) continue;
    atomicMin(&best[run_slot * B + 2 * sl], (unsigned long long)run0);
    atomicMin(&best[run_slot * B + 2 * sl + 1], (unsigned long long)run1);
    uint64_t nb0[NPW / G], nb1[NPW / G];
#pragma unroll
    for (int i = 0; i < NPW / G; i++) {
      nb0[i] = best[(i * G + gh) * B + 2 * sl];
      nb1[i] = best[(i * G + gh) * B + 2 * sl + 1];
    }
    if (!prefetched) {
#pragma unroll
      for (int i = 0; i < NPW / G; i++)
        load_key2(slab,
                  nb0[i] != KEY_INF || nb1[i] != KEY_INF ? min(vw + i * G + gh, vw1 - 1) * (B * 8) + lane16 : OOB,
                  cur0[i], cur1[i]);
    }
    bool any = false;
#pragma unroll
    for (int i = 0; i < NPW / G; i++) {
      const uint32_t v = vw + i * G + gh;
      bool c0 = v < vw1 && nb0[i] < cur0[i];
      bool c1 = v < vw1 && nb1[i] < cur1[i];
      if (nseg > 1) {  // other segments' waves write this row too
        unsigned long long* k = (unsigned long long*)&Db[(size_t)v * B + 2 * sl];
        if (c0) c0 = nb0[i] < atomicMin(k, (unsigned long long)nb0[i]);
        if (c1) c1 = nb1[i] < atomicMin(k + 1, (unsigned long long)nb1[i]);
      } else if (c0 || c1) {
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        *(u64x2*)&Db[(size_t)v * B + 2 * sl] = (u64x2){c0 ? nb0[i] : cur0[i], c1 ? nb1[i] : cur1[i]};
      }
      const uint64_t m = __ballot(c0 || c1);
      if (m) {
        any = true;
        if (FRONT && sl == 0 && ((m >> (gh * LPR)) & ROW_MASK)) stamp[(size_t)b * n + v] = pass + 2;
      }
    }
    if (any && b != flagged) {
      if (lane == 0) changed[b * FLAG_STRIDE] = 1u;
      flagged = b;
    }
  }
  if (COUNT && lane == 0 && n_rel) atomicAdd(&work[blockIdx.x & (WORK_SHARDS - 1)], (unsigned long long)n_rel * B);
}

// Transposed write-out of [B rows x 64 cols] tiles.  Diagonal = the raw
// self-loop (graph/mod.rs:210-217).  Saturated keys flag their batch.
// VEC: 16-B stores (two latencies / four losses per lane); needs n_used % 4 == 0
// so every row starts 16-B aligned.
__device__ __forceinline__ void out_entry(uint64_t kk, uint32_t row, uint32_t j, const uint32_t* __restrict__ used,
                                          const uint32_t* __restrict__ self_edge, const uint64_t* __restrict__ e_lat,
                                          const float* __restrict__ e_loss, uint64_t& lat, float& loss, bool& sflag) {
  if (row == j) {
    const uint32_t e = self_edge[used[j]];
    lat = e_lat[e];
    loss = e_loss[e];
  } else {
    const uint32_t l = key_lat(kk);
    sflag |= l == LAT32_SAT;
    lat = l;
    loss = __uint_as_float(key_loss_bits(kk));
  }
}

// TPB column tiles per block: the global loads of tile t + 1 are issued into
// registers before tile t is written out, so a block's reads and writes overlap.
template <int B, bool VEC, int TPB>
__global__ void __launch_bounds__(256)
    k_out_batch(const uint64_t* __restrict__ D, uint32_t n, const uint32_t* __restrict__ used, uint32_t n_used,
                uint32_t first_row, uint32_t row_end, uint32_t out_row0, const uint32_t* __restrict__ self_edge,
                const uint64_t* __restrict__ e_lat, const float* __restrict__ e_loss,
                uint64_t* __restrict__ out_lat, float* __restrict__ out_loss, uint32_t* __restrict__ sat) {
  constexpr int G = 64 / B;
  constexpr int CPW = 64 / (4 * G);  // tile columns (nodes) each lane loads
  __shared__ uint64_t tile[64][B + 1];
  const uint32_t b = blockIdx.y;
  const uint64_t* __restrict__ Db = D + (size_t)b * n * B;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int gh = lane / B, sl = lane % B;
  uint64_t pre[CPW];
  auto load_tile = [&](uint32_t j0) {
    uint32_t node[CPW];
#pragma unroll
    for (int k = 0; k < CPW; k++) {
      const uint32_t j = j0 + wave * G + gh + k * 4 * G;
      node[k] = j < n_used ? used[j] : ~0u;
    }
#pragma unroll
    for (int k = 0; k < CPW; k++) pre[k] = node[k] != ~0u ? Db[(size_t)node[k] * B + sl] : 0ull;
  };
  bool sflag = false;
  const uint32_t rbase = first_row + b * B;
  const uint32_t jb = blockIdx.x * TPB * 64;
  load_tile(jb);
  for (int t = 0; t < TPB; t++) {
    const uint32_t j0 = jb + t * 64;
    if (j0 >= n_used) break;
    if (t) __syncthreads();  // the previous tile's write-out has read the LDS tile
#pragma unroll
    for (int k = 0; k < CPW; k++) tile[wave * G + gh + k * 4 * G][sl] = pre[k];
    __syncthreads();
    if (t + 1 < TPB && j0 + 64 < n_used) load_tile(j0 + 64);
    if (VEC && j0 + 64 <= n_used) {
      // lane = (row quarter, 4 columns): each key is read from LDS once, and the
      // lane stores 32 B of latencies and 16 B of losses
      for (int r = wave * 4 + (lane >> 4); r < B; r += 16) {
        const uint32_t row = rbase + r;
        if (row >= row_end) continue;
        const uint32_t c = (lane & 15) * 4;
        uint64_t l0, l1, l2, l3;
        float4 f;
        out_entry(tile[c][r], row, j0 + c, used, self_edge, e_lat, e_loss, l0, f.x, sflag);
        out_entry(tile[c + 1][r], row, j0 + c + 1, used, self_edge, e_lat, e_loss, l1, f.y, sflag);
        out_entry(tile[c + 2][r], row, j0 + c + 2, used, self_edge, e_lat, e_loss, l2, f.z, sflag);
        out_entry(tile[c + 3][r], row, j0 + c + 3, used, self_edge, e_lat, e_loss, l3, f.w, sflag);
        const size_t o = (size_t)(row - out_row0) * n_used + j0 + c;
        // write-once streaming output (1.2 GB at 10k): nontemporal 16-B stores
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        typedef float f32x4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store((u64x2){l0, l1}, (u64x2*)&out_lat[o]);
        __builtin_nontemporal_store((u64x2){l2, l3}, (u64x2*)&out_lat[o + 2]);
        __builtin_nontemporal_store((f32x4){f.x, f.y, f.z, f.w}, (f32x4*)&out_loss[o]);
      }
    } else {
      const uint32_t j = j0 + lane;
      for (int r = wave; r < B; r += 4) {
        const uint32_t row = rbase + r;
        if (row >= row_end || j >= n_used) continue;
        const size_t o = (size_t)(row - out_row0) * n_used + j;
        uint64_t l;
        float f;
        out_entry(tile[lane][r], row, j, used, self_edge, e_lat, e_loss, l, f, sflag);
        out_lat[o] = l;
        out_loss[o] = f;
      }
    }
  }
  if (__any(sflag) && lane == 0) atomicOr(&sat[b], 1u);
}

// ---------------------------------------------------------------------------
// Wide fallback: u64 latency + f32 loss, Jacobi (double-buffered) so a reader
// never sees a torn pair.  UINT64_MAX latency = no path yet.
// ---------------------------------------------------------------------------
__global__ void k_init_wide(uint64_t* __restrict__ L, float* __restrict__ F, uint32_t n,
                            const uint32_t* __restrict__ used, const uint32_t* __restrict__ rows,
                            uint32_t n_rows_total, uint32_t n_batches) {
  size_t total = (size_t)n_batches * n * BATCH;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    uint32_t lane = (uint32_t)(i & (BATCH - 1));
    size_t bv = i / BATCH;
    uint32_t v = (uint32_t)(bv % n);
    uint32_t b = (uint32_t)(bv / n);
    uint32_t slot = b * BATCH + lane;
    bool src = slot < n_rows_total && used[rows[slot]] == v;
    L[i] = src ? 0ull : ~0ull;
    F[i] = 0.0f;
  }
}

__global__ void __launch_bounds__(RELAX_BLOCK)
    k_relax_wide(const uint32_t* __restrict__ in_off, const uint32_t* __restrict__ in_src,
                 const uint64_t* __restrict__ in_lat, const float* __restrict__ in_om,
                 const uint64_t* __restrict__ Lc, const float* __restrict__ Fc,
                 uint64_t* __restrict__ Ln, float* __restrict__ Fn, uint32_t n,
                 uint32_t* __restrict__ changed) {
  const uint32_t b = blockIdx.y;
  const size_t base = (size_t)b * n * BATCH;
  const int lane = threadIdx.x & 63;
  const uint32_t v = __builtin_amdgcn_readfirstlane(blockIdx.x * RELAX_WAVES + (threadIdx.x >> 6));
  if (v >= n) return;
  uint64_t bl = Lc[base + (size_t)v * BATCH + lane];
  float bf = Fc[base + (size_t)v * BATCH + lane];
  const uint64_t l_in = bl;
  const float f_in = bf;
  for (uint32_t a = in_off[v]; a < in_off[v + 1]; a++) {
    uint32_t u = in_src[a];
    uint64_t lu = Lc[base + (size_t)u * BATCH + lane];
    if (lu == ~0ull) continue;
    float fu = Fc[base + (size_t)u * BATCH + lane];
    uint64_t cl = lu + in_lat[a];
    float cf = fold_loss(fu, in_om[a]);
    if (cl < bl || (cl == bl && cf < bf)) {
      bl = cl;
      bf = cf;
    }
  }
  Ln[base + (size_t)v * BATCH + lane] = bl;
  Fn[base + (size_t)v * BATCH + lane] = bf;
  bool ch = bl != l_in || __float_as_uint(bf) != __float_as_uint(f_in);
  if (__any(ch) && lane == 0) *changed = 1u;  // plain store: the line stays in L2
}

__global__ void k_out_wide(const uint64_t* __restrict__ L, const float* __restrict__ F, uint32_t n,
                           const uint32_t* __restrict__ used, uint32_t n_used,
                           const uint32_t* __restrict__ rows, uint32_t n_rows_total, uint32_t out_row0,
                           const uint32_t* __restrict__ self_edge, const uint64_t* __restrict__ e_lat,
                           const float* __restrict__ e_loss, uint64_t* __restrict__ out_lat,
                           float* __restrict__ out_loss, unsigned long long* __restrict__ first_unreach) {
  const uint32_t slot = blockIdx.y * BATCH + (threadIdx.x & 63);
  if (slot >= n_rows_total) return;
  const uint32_t row = rows[slot];
  const size_t base = (size_t)blockIdx.y * n * BATCH + (threadIdx.x & 63);
  for (uint32_t j = blockIdx.x * 4 + (threadIdx.x >> 6); j < n_used; j += gridDim.x * 4) {
    size_t o = (size_t)(row - out_row0) * n_used + j;
    if (row == j) {
      uint32_t e = self_edge[used[j]];
      out_lat[o] = e_lat[e];
      out_loss[o] = e_loss[e];
      continue;
    }
    uint64_t l = L[base + (size_t)used[j] * BATCH];
    out_lat[o] = l;
    out_loss[o] = F[base + (size_t)used[j] * BATCH];
    if (l == ~0ull) atomicMin(first_unreach, (unsigned long long)row * n_used + j);
  }
}

// ---------------------------------------------------------------------------
// Self-loop census over the used nodes (graph/mod.rs:210-217): first failing
// node in order, low bit = "more than one".
// ---------------------------------------------------------------------------
__global__ void k_self_check(const uint32_t* __restrict__ used, uint32_t n_used,
                             const uint32_t* __restrict__ self_cnt,
                             unsigned long long* __restrict__ first) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n_used; j += gridDim.x * blockDim.x) {
    uint32_t c = self_cnt[used[j]];
    if (c != 1) atomicMin(first, ((unsigned long long)j << 1) | (c > 1 ? 1ull : 0ull));
  }
}

// The LDS search's last launch of a build: how many rows it flagged for the wide
// kernel, and (when sg_routing_build asked for it) the self-loop check's first
// failure as k_self_check encodes it, both into the mapped return block -- the
// build's end is one synchronisation and no copies.  One workgroup, branch-free loads.
__global__ void __launch_bounds__(1024) k_build_finish(const uint32_t* __restrict__ sat, uint32_t rows,
                                                       const uint32_t* __restrict__ used, uint32_t n_used,
                                                       const uint32_t* __restrict__ self_cnt, uint32_t* __restrict__ ret) {
  constexpr int G = 8;
  __shared__ uint32_t s_cnt[16];
  __shared__ unsigned long long s_min[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr uint32_t OOB = 0x80000000u;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)sat, 0, (int)(rows * 4u), 0x00020000);
  uint32_t cnt = 0;
  for (uint32_t r0 = tid; r0 < rows; r0 += G * 1024) {
    uint32_t x[G];
#pragma unroll
    for (int g = 0; g < G; g++) {
      const uint32_t r = r0 + g * 1024;
      x[g] = __builtin_amdgcn_raw_buffer_load_b32(rs, r < rows ? r * 4u : OOB, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < G; g++) cnt += x[g] != 0u;
  }
  unsigned long long first = ~0ull;
  if (self_cnt) {
    const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc((void*)used, 0, (int)(n_used * 4u), 0x00020000);
    for (uint32_t j0 = tid; j0 < n_used; j0 += G * 1024) {
      uint32_t v[G], c[G];
#pragma unroll
      for (int g = 0; g < G; g++) {
        const uint32_t j = j0 + g * 1024;
        v[g] = __builtin_amdgcn_raw_buffer_load_b32(ru, j < n_used ? j * 4u : OOB, 0, 0);
      }
#pragma unroll
      for (int g = 0; g < G; g++) c[g] = j0 + g * 1024 < n_used ? self_cnt[v[g]] : 1u;
#pragma unroll
      for (int g = 0; g < G; g++)
        if (c[g] != 1u) first = min(first, ((unsigned long long)(j0 + g * 1024) << 1) | (c[g] > 1u ? 1ull : 0ull));
    }
  }
  cnt = wave_incl_sum(cnt);
  for (int d = 32; d > 0; d >>= 1) first = min(first, (unsigned long long)__shfl_xor(first, d));
  if (lane == 63) s_cnt[wv] = cnt;
  if (lane == 0) s_min[wv] = first;
  __syncthreads();
  if (tid == 0) {
    uint32_t t = 0;
    unsigned long long m = ~0ull;
    for (int w = 0; w < 16; w++) {
      t += s_cnt[w];
      m = min(m, s_min[w]);
    }
    ret[4] = t;
    ((unsigned long long*)ret)[1] = m;
  }
}

// ---------------------------------------------------------------------------
// Direct paths (graph/mod.rs:230-252): per used pair, count the edges that
// petgraph's edges_connecting would yield.
// ---------------------------------------------------------------------------
__global__ void k_pair_count(const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                             uint32_t m, int directed, const uint32_t* __restrict__ map,
                             uint32_t n_used, uint32_t row_begin, uint32_t row_end,
                             uint32_t* __restrict__ cnt, uint32_t* __restrict__ edge) {
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < m; e += gridDim.x * blockDim.x) {
    uint32_t iu = map[src[e]], iv = map[dst[e]];
    if (iu == ~0u || iv == ~0u) continue;
    if (iu >= row_begin && iu < row_end) {
      size_t o = (size_t)(iu - row_begin) * n_used + iv;
      atomicAdd(&cnt[o], 1u);
      edge[o] = e;
    }
    if (!directed && iu != iv && iv >= row_begin && iv < row_end) {
      size_t o = (size_t)(iv - row_begin) * n_used + iu;
      atomicAdd(&cnt[o], 1u);
      edge[o] = e;
    }
  }
}

__global__ void k_pair_out(const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ edge,
                           size_t count, uint32_t n_used, uint32_t row_begin,
                           const uint64_t* __restrict__ e_lat, const float* __restrict__ e_loss,
                           uint64_t* __restrict__ out_lat, float* __restrict__ out_loss,
                           unsigned long long* __restrict__ first) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
       i += (size_t)gridDim.x * blockDim.x) {
    uint32_t c = cnt[i];
    if (c != 1) {
      unsigned long long lin = (unsigned long long)row_begin * n_used + i;
      atomicMin(first, (lin << 1) | (c > 1 ? 1ull : 0ull));
      out_lat[i] = 0;
      out_loss[i] = 0.0f;
    } else {
      out_lat[i] = e_lat[edge[i]];
      out_loss[i] = e_loss[edge[i]];
    }
  }
}

// Two-stage minimum: per-block partials (plain stores), then one block.
__global__ void __launch_bounds__(256) k_min_u64(const uint64_t* __restrict__ x, size_t count,
                                                 unsigned long long* __restrict__ part) {
  __shared__ unsigned long long wm[4];
  unsigned long long m = ~0ull;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x)
    m = min(m, (unsigned long long)x[i]);
  for (int d = 32; d > 0; d >>= 1) m = min(m, (unsigned long long)__shfl_xor(m, d, 64));
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = min(min(wm[0], wm[1]), min(wm[2], wm[3]));
}

__global__ void __launch_bounds__(256) k_min_final(const unsigned long long* __restrict__ part, uint32_t n,
                                                   unsigned long long* __restrict__ out) {
  __shared__ unsigned long long wm[4];
  unsigned long long m = ~0ull;
  for (uint32_t i = threadIdx.x; i < n; i += 256) m = min(m, part[i]);
  for (int d = 32; d > 0; d >>= 1) m = min(m, (unsigned long long)__shfl_xor(m, d, 64));
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) *out = min(min(wm[0], wm[1]), min(wm[2], wm[3]));
}

// sg_routing_info_fill: a block of (latency u64, loss f32) cells -> the host
// RoutingInfo's 8-byte cells (latency u32 << 32 | bits(loss); SG_CELL_WIDE in the
// latency half when the path takes 2^32 - 1 ns or more), the block's smallest
// latency (ctl[0], atomicMin) and its count of wide cells (ctl[1]).
__global__ void __launch_bounds__(256) k_pack_cells(const uint64_t* __restrict__ lat, const float* __restrict__ loss,
                                                    size_t cells, uint64_t* __restrict__ out,
                                                    unsigned long long* __restrict__ ctl) {
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  unsigned long long m = ~0ull;
  uint32_t nw = 0;
  auto pack = [&](uint64_t l, float f) -> uint64_t {
    m = min(m, (unsigned long long)l);
    const uint32_t hi = l < SG_CELL_WIDE ? (uint32_t)l : SG_CELL_WIDE;
    nw += hi == SG_CELL_WIDE;
    return ((uint64_t)hi << 32) | __float_as_uint(f);
  };
  const size_t pairs = cells / 2, stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < pairs; i += stride) {
    const u64x2 l = __builtin_nontemporal_load((const u64x2*)lat + i);
    const f32x2 f = __builtin_nontemporal_load((const f32x2*)loss + i);
    __builtin_nontemporal_store((u64x2){pack(l.x, f.x), pack(l.y, f.y)}, (u64x2*)out + i);
  }
  if ((cells & 1) && blockIdx.x == 0 && threadIdx.x == 0) out[cells - 1] = pack(lat[cells - 1], loss[cells - 1]);
  for (int d = 32; d > 0; d >>= 1) {
    m = min(m, (unsigned long long)__shfl_xor(m, d, 64));
    nw += __shfl_xor(nw, d, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (m != ~0ull) atomicMin(&ctl[0], m);
    if (nw) atomicAdd(&ctl[1], (unsigned long long)nw);
  }
}

// the wide cells of a block: (cell index + off, u64 latency) pairs, in any order
__global__ void k_wide_list(const uint64_t* __restrict__ lat, size_t cells, uint64_t off,
                            unsigned long long* __restrict__ ctr, uint64_t* __restrict__ list) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells; i += stride)
    if (lat[i] >= SG_CELL_WIDE) {
      const unsigned long long k = atomicAdd(ctr, 1ull);
      list[2 * k] = off + i;
      list[2 * k + 1] = lat[i];
    }
}

// Diagnostics only (SG_PLAN_WARM): keep every CU busy for `iters` dependent
// VALU steps, to tell clock ramp-up from kernel cost in A/B runs.
__global__ void k_busy(uint32_t iters, float* __restrict__ sink) {
  float x = threadIdx.x * 1e-3f;
  for (uint32_t i = 0; i < iters; i++) x = x * 0.999f + 1e-4f;
  if (x == 12345.0f) sink[0] = x;
}

// ---------------------------------------------------------------------------
// Host orchestration
// ---------------------------------------------------------------------------
static std::string node_name(const sg_net* net, uint32_t idx) {
  uint32_t id = net->gml_id.empty() ? idx : net->gml_id[idx];
  return std::to_string(id);
}

static int env_int(const char* name, int dflt) {
  const char* s = getenv(name);
  return s && *s ? atoi(s) : dflt;
}

template <class T>
static T* dmalloc(size_t count) {
  void* p = nullptr;
  SG_HIP(hipMalloc(&p, std::max<size_t>(count * sizeof(T), 16)));
  return static_cast<T*>(p);
}

// A fresh network per simulation (the reference builds its graph once and computes
// the table once, sim_config.rs:76-79, :137-141): one device allocation for every
// array, the arc count from the host edge list (no device round trip), and no
// stream synchronisation -- the build that follows orders after these launches.
static void build_net(sg_ctx* ctx, const sg_graph* g, sg_net* net) {
  const uint32_t n = g->n_nodes, m = g->n_edges;
  if (m && (!g->edge_src || !g->edge_dst || !g->edge_latency_ns || !g->edge_packet_loss))
    throw Error(SG_ERR_INVALID_ARG, "null edge array");
  // Validation, in branch-free passes over the edge arrays (part of every one-shot
  // build).  One thread: the endpoints (and the self-loop count the sizes need) before
  // anything is allocated, the losses and latencies, which index nothing, after the
  // upload's launches, while the device runs them.  Large lists: every check in the
  // threaded staging pass below, before any launch.  Either way a bad edge is named by
  // the per-edge loop, which checks every rule edge by edge (the reference's order).
  const uint32_t* __restrict__ es = g->edge_src;
  const uint32_t* __restrict__ ed = g->edge_dst;
  const uint64_t* __restrict__ el = g->edge_latency_ns;
  const float* __restrict__ ef = g->edge_packet_loss;
  const bool trace = env_int("SG_NET_TRACE", 0) != 0;  // (diagnostics: host phases on stderr)
  auto now_us = []() {
    return (double)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count() / 1e3;
  };
  const double tr0 = trace ? now_us() : 0.0;
  double tr[6] = {0, 0, 0, 0, 0, 0};
  auto name_bad_edge = [&]() {
    for (uint32_t e = 0; e < m; e++) {
      if (es[e] >= n || ed[e] >= n)
        throw Error(SG_ERR_INVALID_ARG, "edge " + std::to_string(e) + " endpoint out of range");
      const float l = ef[e];
      if (!(l >= 0.0f && l <= 1.0f))  // graph/mod.rs:101-103 (NaN rejected too)
        throw Error(SG_ERR_INVALID_ARG, "Edge 'packet_loss' is not in the range [0,1]");
      if (el[e] == 0)  // graph/mod.rs:105-107
        throw Error(SG_ERR_INVALID_ARG, "Edge 'latency' must not be 0");
    }
  };
  // one allocation, 256-B aligned sub-arrays; the edge arrays first (their offsets depend on m
  // only, so they can be staged before the self-loop count sizes the rest)
  size_t total = 0;
  // (SG_NET_ALIGN, A/B diagnostics: sub-array alignment in bytes)
  const size_t align = (size_t)std::max(256, env_int("SG_NET_ALIGN", 256));
  auto carve = [&](size_t bytes) {
    const size_t o = total;
    total += (std::max<size_t>(bytes, 16) + align - 1) / align * align;
    return o;
  };
  const size_t o_esrc = carve(m * 4ull), o_edst = carve(m * 4ull), o_elat = carve(m * 8ull),
               o_eloss = carve(m * 4ull);
  const size_t eb = total;  // bytes of the edge arrays, up to the first derived array
  // Large edge lists (C2's 720k edges): validation and the copy into the pinned staging over
  // up to 4 host threads (one thread 349 us, 4 threads 134 us on the MI355X box's host;
  // tools/debug/stage_thread_probe.cpp), in two parts, each DMA'd as soon as it is staged:
  // (A) the endpoints -- checked, self-loops counted -- then (B) the latencies and losses --
  // checked -- while A's DMA runs.  The block is sized for no self-loops, since it is allocated
  // before the count is known (the arrays then have a little unused room).  Small lists
  // (C3's 50k edges: 22 us) take one thread, where the threads' start-up costs more than they
  // save, and check the losses and latencies after the upload's launches.
  // (SG_NET_THREADS: A/B diagnostics, 1 = one thread)
  const uint64_t arcs_cap = (uint64_t)m * (g->directed ? 1u : 2u);
  const uint32_t n_thr = m >= (1u << 18) && arcs_cap < (1ull << 32)
                             ? (uint32_t)std::max(1, std::min(4, env_int("SG_NET_THREADS", 4)))
                             : 1u;
  const bool threaded = n_thr > 1;
  uint64_t n_self = 0;
  if (!threaded) {
    uint32_t bad = 0, ns = 0;
    for (uint32_t e = 0; e < m; e++) {
      const uint32_t a = es[e], b = ed[e];
      bad |= (uint32_t)(a >= n) | (uint32_t)(b >= n);
      ns += a == b;
    }
    if (bad) name_bad_edge();
    n_self = ns;
  }
  if (trace) tr[0] = now_us();
  // arcs without self-loops, both directions when undirected (petgraph semantics, graph/mod.rs:137-152)
  const uint64_t arcs_sz = threaded ? arcs_cap : ((uint64_t)m - n_self) * (g->directed ? 1u : 2u);
  if (arcs_sz >= (1ull << 32)) throw Error(SG_ERR_INVALID_ARG, "too many arcs");
  const uint32_t n_arcs_sz = (uint32_t)arcs_sz;  // the layout's arc count (an upper bound when threaded)
  net->ctx = ctx;
  net->n_nodes = n;
  net->n_edges = m;
  net->directed = g->directed != 0;
  if (g->node_gml_id) net->gml_id.assign(g->node_gml_id, g->node_gml_id + n);
  hipStream_t st = ctx->stream;
  const size_t o_inoff = carve(((size_t)n + 1) * 4), o_scnt = carve((size_t)n * 4),
               o_sedge = carve((size_t)n * 4), o_insrc = carve(n_arcs_sz * 4ull),
               o_inlat = carve(n_arcs_sz * 8ull), o_inom = carve(n_arcs_sz * 4ull),
               o_inrec = carve(n_arcs_sz * 16ull), o_outoff = carve(((size_t)n + 1) * 4),
               o_outarc = carve(n_arcs_sz * 12ull);
  {  // a released block of the right size from the context's pool, else a new one
    size_t best = ~(size_t)0;
    for (size_t i = 0; i < ctx->net_pool.size(); i++) {
      const size_t b = ctx->net_pool[i].bytes;
      if (b >= total && b <= 2 * total + (1u << 20) && (best == ~(size_t)0 || b < ctx->net_pool[best].bytes)) best = i;
    }
    if (best != ~(size_t)0) {
      auto blk = ctx->net_pool[best];
      ctx->net_pool.erase(ctx->net_pool.begin() + best);
      SG_HIP(hipStreamWaitEvent(ctx->stream, blk.freed, 0));
      (void)hipEventDestroy(blk.freed);
      net->mem = blk.p;
      net->mem_bytes = blk.bytes;
    } else {
      SG_HIP(hipMalloc(&net->mem, total));
      net->mem_bytes = total;
    }
  }
  if (trace) tr[1] = now_us();
  char* base = (char*)net->mem;
  net->e_src = (uint32_t*)(base + o_esrc);
  net->e_dst = (uint32_t*)(base + o_edst);
  net->e_lat = (uint64_t*)(base + o_elat);
  net->e_loss = (float*)(base + o_eloss);
  net->in_off = (uint32_t*)(base + o_inoff);
  net->self_cnt = (uint32_t*)(base + o_scnt);
  net->self_edge = (uint32_t*)(base + o_sedge);
  net->in_src = (uint32_t*)(base + o_insrc);
  net->in_lat = (uint64_t*)(base + o_inlat);
  net->in_om = (float*)(base + o_inom);
  net->in_rec = (uint4*)(base + o_inrec);
  net->out_off = (uint32_t*)(base + o_outoff);
  net->out_arc = (uint32_t*)(base + o_outarc);
  // a bad edge found once the block is allocated: nothing may still run on the block when
  // the caller deletes the net, then the per-edge loop names it
  auto reject = [&]() {
    (void)hipStreamSynchronize(st);
    (void)hipFree(net->mem);
    net->mem = nullptr;
    name_bad_edge();
  };
  bool checked = false;  // losses and latencies checked (threaded: in part B)
  if (threaded) {
    char* staged = stage_acquire(ctx, 0, eb);
    std::vector<uint32_t> bad_t(n_thr, 0u), ns_t(n_thr, 0u);
    std::atomic<uint32_t> done_a{0u}, done_b{0u};
    auto range = [&](uint32_t t, uint32_t& e0, uint32_t& e1) {
      e0 = (uint32_t)((uint64_t)m * t / n_thr);
      e1 = (uint32_t)((uint64_t)m * (t + 1) / n_thr);
    };
    auto part_a = [&](uint32_t t) {  // endpoints: checked, self-loops counted, staged
      uint32_t e0, e1, bad = 0, ns = 0;
      range(t, e0, e1);
      for (uint32_t e = e0; e < e1; e++) {
        const uint32_t a = es[e], b = ed[e];
        bad |= (uint32_t)(a >= n) | (uint32_t)(b >= n);
        ns += a == b;
      }
      memcpy(staged + o_esrc + e0 * 4ull, es + e0, (e1 - e0) * 4ull);
      memcpy(staged + o_edst + e0 * 4ull, ed + e0, (e1 - e0) * 4ull);
      bad_t[t] = bad;
      ns_t[t] = ns;
      done_a.fetch_add(1u, std::memory_order_release);
    };
    auto part_b = [&](uint32_t t) {  // losses and latencies: checked, staged
      uint32_t e0, e1, bad = 0;
      range(t, e0, e1);
      for (uint32_t e = e0; e < e1; e++) bad |= (uint32_t)!(ef[e] >= 0.0f) | (uint32_t)!(ef[e] <= 1.0f);
      for (uint32_t e = e0; e < e1; e++) bad |= (uint32_t)(el[e] == 0);
      memcpy(staged + o_elat + e0 * 8ull, el + e0, (e1 - e0) * 8ull);
      memcpy(staged + o_eloss + e0 * 4ull, ef + e0, (e1 - e0) * 4ull);
      bad_t[t] |= bad;
      done_b.fetch_add(1u, std::memory_order_release);
    };
    std::vector<std::thread> pool;
    struct Joiner {  // every started thread is joined, whatever is thrown below
      std::vector<std::thread>& p;
      ~Joiner() {
        for (auto& th : p)
          if (th.joinable()) th.join();
      }
    } joiner{pool};
    uint32_t started = 1;  // threads 1 .. started-1 run their parts; this thread runs the others
    try {
      for (uint32_t t = 1; t < n_thr; t++, started++)
        pool.emplace_back([&, t] {
          part_a(t);
          part_b(t);
        });
    } catch (const std::system_error&) {
    }
    // each part's DMA once every thread has staged it: A's runs while part B is staged
    for (uint32_t t = 0; t < n_thr; t++)
      if (t == 0 || t >= started) part_a(t);
    while (done_a.load(std::memory_order_acquire) < n_thr) std::this_thread::yield();
    const hipError_t ea = hipMemcpyAsync(base, staged, o_elat, hipMemcpyHostToDevice, st);
    for (uint32_t t = 0; t < n_thr; t++)
      if (t == 0 || t >= started) part_b(t);
    while (done_b.load(std::memory_order_acquire) < n_thr) std::this_thread::yield();
    const hipError_t eb2 = ea == hipSuccess ? hipMemcpyAsync(base + o_elat, staged + o_elat, eb - o_elat,
                                                             hipMemcpyHostToDevice, st)
                                            : ea;
    for (auto& th : pool) th.join();
    SG_HIP(eb2);
    stage_release(ctx, 0);
    uint32_t bad = 0;
    for (uint32_t t = 0; t < n_thr; t++) {
      bad |= bad_t[t];
      n_self += ns_t[t];
    }
    if (bad) reject();
    checked = true;
    if (trace) tr[2] = now_us();
  } else if (m) {  // the edge arrays through the context's pinned staging, one copy (they are adjacent)
    char* h = stage_acquire(ctx, 0, eb);
    memcpy(h + o_esrc, g->edge_src, m * 4ull);
    memcpy(h + o_edst, g->edge_dst, m * 4ull);
    memcpy(h + o_elat, g->edge_latency_ns, m * 8ull);
    memcpy(h + o_eloss, g->edge_packet_loss, m * 4ull);
    if (trace) tr[2] = now_us();
    SG_HIP(hipMemcpyAsync(base, h, eb, hipMemcpyHostToDevice, st));
    stage_release(ctx, 0);
  }
  const uint32_t n_arcs = (uint32_t)(((uint64_t)m - n_self) * (g->directed ? 1u : 2u));
  net->n_arcs = n_arcs;
  if (trace) tr[3] = now_us();
  uint32_t* indeg = ctx->r_misc.get<uint32_t>(2 * ((size_t)n + 1));
  uint32_t* outdeg = indeg + n + 1;
  // the degree counters, and self_cnt with self_edge (adjacent): self_edge stays 0 where no
  // self-loop sets it, so a build that reads it before the self-loop check's error is raised
  // stays in bounds
  {
    const uint32_t na = 2 * (n + 1), nb = (uint32_t)((o_insrc - o_scnt) / 4);
    hipLaunchKernelGGL(k_zero2, dim3(grid_for((size_t)na + nb, 256, 1024)), dim3(256), 0, st, indeg, na,
                       net->self_cnt, nb);
    SG_CHECK_LAUNCH();
  }
  const bool lds_up = n <= NET_LDS_NODES && env_int("SG_NET_LDS", 1) != 0;  // (SG_NET_LDS=0: A/B)
  const uint32_t lds_blocks = std::max(1u, std::min(NET_LDS_BLOCKS, (m + 255) / 256));
  if (m) {
    if (lds_up)
      hipLaunchKernelGGL(k_net_count_lds, dim3(lds_blocks), dim3(256), 0, st, net->e_src, net->e_dst, m, n,
                         (int)net->directed, indeg, outdeg, net->self_cnt, net->self_edge);
    else
      hipLaunchKernelGGL(k_net_count, dim3(grid_for(m, 256, 8192)), dim3(256), 0, st, net->e_src, net->e_dst, m,
                         (int)net->directed, indeg, outdeg, net->self_cnt, net->self_edge);
    SG_CHECK_LAUNCH();
  }
  uint32_t* cursor = ctx->r_map.get<uint32_t>(2 * ((size_t)n + 1));
  uint32_t* ocursor = cursor + n + 1;
  if (n < NET_SCAN_SMALL) {
    hipLaunchKernelGGL(k_net_scan, dim3(1), dim3(1024), 0, st, indeg, outdeg, n, net->in_off, cursor, net->out_off,
                       ocursor);
    SG_CHECK_LAUNCH();
  } else {
    exclusive_scan_u32(ctx, indeg, net->in_off, n);
    exclusive_scan_u32(ctx, outdeg, net->out_off, n);
    SG_HIP(hipMemcpyAsync(cursor, net->in_off, ((size_t)n + 1) * 4, hipMemcpyDeviceToDevice, st));
    SG_HIP(hipMemcpyAsync(ocursor, net->out_off, ((size_t)n + 1) * 4, hipMemcpyDeviceToDevice, st));
  }
  if (n_arcs) {
    // the out-arcs only; the in-arcs wait for a search that reads them (ensure_csc)
    if (lds_up)
      hipLaunchKernelGGL((k_net_scatter_lds<true, false>), dim3(lds_blocks), dim3(256), 0, st, net->e_src, net->e_dst,
                         net->e_lat, net->e_loss, m, n, (int)net->directed, cursor, net->in_src, net->in_lat,
                         net->in_om, net->in_rec, ocursor, net->out_arc);
    else
      hipLaunchKernelGGL((k_net_scatter<true, false>), dim3(grid_for(m, 256, 8192)), dim3(256), 0, st, net->e_src,
                         net->e_dst, net->e_lat, net->e_loss, m, (int)net->directed, cursor, net->in_src, net->in_lat,
                         net->in_om, net->in_rec, ocursor, net->out_arc);
    SG_CHECK_LAUNCH();
  }
  {  // the losses and latencies, while the device runs the upload (threaded: checked already)
    uint32_t bad = 0;
    if (!checked) {
      for (uint32_t e = 0; e < m; e++) bad |= (uint32_t)!(ef[e] >= 0.0f) | (uint32_t)!(ef[e] <= 1.0f);
      for (uint32_t e = 0; e < m; e++) bad |= (uint32_t)(el[e] == 0);
    }
    // the arcs' latency statistics the bucketed search sizes its buckets from (graphs past the
    // LDS search, or SG_APSP_BUCKET=1): smallest and mean arc latency, self-loops excluded
    if (!bad && (!sssp_lds_fits(n) || env_int("SG_APSP_BUCKET", -1) == 1)) {
      uint64_t lo = LAT32_SAT;
      double sum = 0.0;
      uint64_t cnt = 0;
      for (uint32_t e = 0; e < m; e++) {
        if (es[e] == ed[e]) continue;
        const uint64_t l = std::min<uint64_t>(el[e], LAT32_SAT);
        lo = std::min(lo, l);
        sum += (double)l;
        cnt++;
      }
      net->arc_lat_min = (uint32_t)lo;
      net->arc_lat_mean = cnt ? sum / (double)cnt : 0.0;
    }
    if (trace) {
      tr[4] = now_us();
      fprintf(stderr, "[net] m=%u: endpoint check %.1f us, allocation %.1f, staging copy %.1f, H2D enqueue %.1f, "
              "kernels enqueue + loss/latency check %.1f\n", m, tr[0] - tr0, tr[1] - tr[0], tr[2] - tr[1],
              tr[3] - tr[2], tr[4] - tr[3]);
    }
    if (bad) reject();
  }
}

// The self-loop check of every used node (graph/mod.rs:210-217) runs ahead of the
// search without a host round trip; its result is read once the build has
// synchronised (raise_self_loops), and an error found there wins over any the
// search raised, as in the reference, where the self-loops are checked before the
// n^2 assertion (:219).  The search reads self_edge only at count 1 (and it is
// zeroed elsewhere), so it stays in bounds on a graph the check rejects.
static unsigned long long* launch_self_loops(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used) {
  unsigned long long* first = ctx->r_self.get<unsigned long long>(4);  // (its own word: the build uses r_err)
  SG_HIP(hipMemsetAsync(first, 0xff, 8, ctx->stream));
  hipLaunchKernelGGL(k_self_check, dim3(grid_for(n_used, 256, 4096)), dim3(256), 0, ctx->stream,
                     d_used, n_used, net->self_cnt, first);
  SG_CHECK_LAUNCH();
  return first;
}

static void raise_self_value(sg_net* net, unsigned long long h, const uint32_t* h_used) {
  if (h != ~0ull) {
    uint32_t j = (uint32_t)(h >> 1);
    std::string id = node_name(net, h_used[j]);
    if (h & 1)
      throw Error(SG_ERR_MULTI_EDGE, "More than one edge connecting node " + id + " to " + id, j, j);
    throw Error(SG_ERR_NO_EDGE, "No edge connecting node " + id + " to " + id, j, j);
  }
}

static void raise_self_loops(sg_ctx* ctx, sg_net* net, const unsigned long long* first, const uint32_t* h_used) {
  unsigned long long h = 0;
  copy_to_host(ctx, &h, first, 8);
  raise_self_value(net, h, h_used);
}

// sg_routing_build's check: the value the LDS search's final kernel read, else a launch of its own
static void raise_self_check(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used,
                             const uint32_t* h_used) {
  const bool done = ctx->self_done;
  const unsigned long long v = ctx->self_first;
  ctx->self_used = nullptr;
  ctx->self_cnt = nullptr;
  ctx->self_done = false;
  if (done) raise_self_value(net, v, h_used);
  else raise_self_loops(ctx, net, launch_self_loops(ctx, net, d_used, n_used), h_used);
}

// Wide recomputation of the listed rows (absolute row indices).
// The in-arc CSC (in_src, in_lat, in_om, in_rec), built on its first use: the scatter again,
// in-arcs only, from cursors set to in_off (the upload's scan wrote it).
void ensure_csc(sg_ctx* ctx, sg_net* net) {
  if (net->csc) return;
  const uint32_t n = net->n_nodes, m = net->n_edges;
  if (net->n_arcs) {
    hipStream_t st = ctx->stream;
    uint32_t* cursor = ctx->r_map.get<uint32_t>((size_t)n + 1);
    SG_HIP(hipMemcpyAsync(cursor, net->in_off, ((size_t)n + 1) * 4, hipMemcpyDeviceToDevice, st));
    if (n <= NET_LDS_NODES && env_int("SG_NET_LDS", 1) != 0)
      hipLaunchKernelGGL((k_net_scatter_lds<false, true>), dim3(std::max(1u, std::min(NET_LDS_BLOCKS, (m + 255) / 256))),
                         dim3(256), 0, st, net->e_src, net->e_dst, net->e_lat, net->e_loss, m, n, (int)net->directed,
                         cursor, net->in_src, net->in_lat, net->in_om, net->in_rec, (uint32_t*)nullptr,
                         (uint32_t*)nullptr);
    else
      hipLaunchKernelGGL((k_net_scatter<false, true>), dim3(grid_for(m, 256, 8192)), dim3(256), 0, st, net->e_src,
                         net->e_dst, net->e_lat, net->e_loss, m, (int)net->directed, cursor, net->in_src,
                         net->in_lat, net->in_om, net->in_rec, (uint32_t*)nullptr, (uint32_t*)nullptr);
    SG_CHECK_LAUNCH();
  }
  net->csc = true;
}

static void run_wide(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used,
                     const std::vector<uint32_t>& rows, uint32_t out_row0, uint64_t* out_lat,
                     float* out_loss) {
  ensure_csc(ctx, net);
  hipStream_t st = ctx->stream;
  const uint32_t n = net->n_nodes;
  const uint32_t nr = (uint32_t)rows.size();
  const uint32_t nb = (nr + BATCH - 1) / BATCH;
  uint32_t* d_rows = ctx->r_misc.get<uint32_t>(nr);
  SG_HIP(hipMemcpyAsync(d_rows, rows.data(), nr * 4ull, hipMemcpyHostToDevice, st));
  size_t slab = (size_t)nb * n * BATCH;
  char* buf = ctx->r_dist2.get<char>(slab * 24);
  uint64_t* L0 = (uint64_t*)buf;
  uint64_t* L1 = L0 + slab;
  float* F0 = (float*)(L1 + slab);
  float* F1 = F0 + slab;
  hipLaunchKernelGGL(k_init_wide, dim3(grid_for(slab, 256, 65536)), dim3(256), 0, st, L0, F0, n,
                     d_used, d_rows, nr, nb);
  uint32_t* changed = ctx->r_flags.get<uint32_t>(4);
  for (uint32_t pass = 0;; pass++) {
    if (pass > n + 2) throw Error(SG_ERR_DEVICE, "wide relaxation did not converge");
    SG_HIP(hipMemsetAsync(changed, 0, 4, st));
    TimedLaunch tl(ctx, "relax_wide", (double)nb * BATCH * net->n_arcs);
    hipLaunchKernelGGL(k_relax_wide, dim3((n + RELAX_WAVES - 1) / RELAX_WAVES, nb), dim3(RELAX_BLOCK),
                       0, st, net->in_off, net->in_src, net->in_lat, net->in_om, L0, F0, L1, F1, n,
                       changed);
    SG_CHECK_LAUNCH();
    std::swap(L0, L1);
    std::swap(F0, F1);
    uint32_t h = 0;
    copy_to_host(ctx, &h, changed, 4);
    if (!h) break;
  }
  unsigned long long* first = ctx->r_err.get<unsigned long long>(4);
  SG_HIP(hipMemsetAsync(first, 0xff, 8, st));
  hipLaunchKernelGGL(k_out_wide, dim3(grid_for(n_used, 4, 1024), nb), dim3(256), 0, st, L0, F0, n,
                     d_used, n_used, d_rows, nr, out_row0, net->self_edge, net->e_lat, net->e_loss,
                     out_lat, out_loss, first);
  SG_CHECK_LAUNCH();
  unsigned long long h = 0;
  copy_to_host(ctx, &h, first, 8);
  if (h != ~0ull) {
    uint32_t i = (uint32_t)(h / n_used), j = (uint32_t)(h % n_used);
    throw Error(SG_ERR_UNREACHABLE, "no path from node index " + std::to_string(i) + " to " +
                                        std::to_string(j) + " (graph must be connected)",
                i, j);
  }
}

// B sources per batch, NPW destination nodes per wave item, STG arcs staged per
// wave step, FRONT = stamp frontier.
template <int B, int NPW, int STG, int GR, bool FRONT, int SPL = 1>
static void shortest_paths_t(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used,
                             uint32_t row_begin, uint32_t row_end, uint64_t* out_lat, float* out_loss) {
  ensure_csc(ctx, net);  // the slab kernel gathers in-arcs
  hipStream_t st = ctx->stream;
  const uint32_t n = net->n_nodes;
  const uint32_t n_rows = row_end - row_begin;
  const uint32_t n_batches = (n_rows + B - 1) / B;
  // slab byte offsets are 32-bit (buffer descriptors; OOB = 0x80000000)
  if ((uint64_t)n * B * 8 >= 0x80000000ull)
    throw Error(SG_ERR_INVALID_ARG, "graph too large for the slab kernel's 32-bit slab offsets (" +
                                        std::to_string(n) + " nodes)");
  // Group: batches whose slabs are live together (bounded device memory).
  const size_t slab_bytes = (size_t)n * B * 8;
  const size_t budget = (size_t)env_int("SG_APSP_GROUP_MB", 4096) << 20;
  const uint32_t group = (uint32_t)std::max<size_t>(1, std::min<size_t>(n_batches, budget / slab_bytes));
  uint64_t* D = ctx->r_dist.get<uint64_t>((size_t)group * n * B);
  uint32_t* stamp = ctx->r_dirty.get<uint32_t>((size_t)group * n);
  // per-batch flags: a 3-slot ring of "changed in pass p" arrays, the
  // saturation flags, the active-batch list
  const size_t fs = (size_t)group * FLAG_STRIDE;
  uint32_t* flags = ctx->r_flags.get<uint32_t>(fs * 3 + 2 * (size_t)group + 8);
  uint32_t* ring[3] = {flags, flags + fs, flags + 2 * fs};
  uint32_t* sat = flags + 3 * fs;
  uint32_t* alist = sat + group;
  unsigned long long* work = ctx->count_work ? ctx->r_work.get<unsigned long long>(WORK_SHARDS) : nullptr;
  if (work) SG_HIP(hipMemsetAsync(work, 0, WORK_SHARDS * 8, st));
  // Passes are issued in chunks; the host reads the convergence flags once per
  // chunk.  A pass issued after its batch converged finds it off the active list.
  const uint32_t chunk = (uint32_t)std::max(1, env_int("SG_APSP_PASS_CHUNK", 4));
  const bool trace = env_int("SG_APSP_TRACE", 0) != 0;  // per-pass diagnostics on stderr
  // in-arc segments per relaxation item (k_relax_w2): one per ~SEG_ARCS arcs of a
  // node chunk, so dense graphs (C2: ~4800 arcs per chunk) fill the chip
  constexpr uint32_t SEG_ARCS = 1200;  // C2 (1,200-node complete graph): 4 segments, measured best (of 1-16)
  const double chunk_arcs = n ? (double)net->n_arcs * NPW / n : 0.0;
  const uint32_t nseg = SPL == 2 ? (uint32_t)std::min(16, std::max(1, env_int("SG_APSP_SEG",
                                       (int)std::lround(chunk_arcs / SEG_ARCS)))) : 1u;
  int out_tpb = env_int("SG_APSP_OUT_TPB", 1);  // column tiles per write-out block: 1 | 2 | 4 (1 measured best)
  out_tpb = out_tpb == 4 ? 4 : out_tpb == 2 ? 2 : 1;
  std::vector<uint32_t> h_sat(group);
  std::vector<uint32_t> wide_rows;
  for (uint32_t g0 = 0; g0 < n_batches; g0 += group) {
    const uint32_t gb = std::min(group, n_batches - g0);
    const uint32_t first_row = row_begin + g0 * B;
    hipLaunchKernelGGL(k_init_batch<B>, dim3(grid_for((size_t)gb * n * (B / 2), 256, 8192)), dim3(256), 0, st, D,
                       stamp, n, gb);
    hipLaunchKernelGGL(k_stamp_sources<B>, dim3(grid_for((size_t)gb * B, 256)), dim3(256), 0, st, D, stamp, n,
                       d_used, first_row, row_end, gb);
    SG_CHECK_LAUNCH();
    SG_HIP(hipMemsetAsync(ring[2], 1, gb * FLAG_STRIDE * 4ull, st));  // "changed in pass -1": every batch active
    // one wave per work item (active batch, NPW-node chunk); 4 waves per block,
    // a multiple of 8 blocks (XCD mapping)
    const uint32_t ncw = (n + 4 * NPW - 1) / (4 * NPW);
    // Sized for the active batches the host last saw (every batch at first; a
    // converged batch never becomes active again, so it is an upper bound for
    // the chunk): a tail pass with few active batches launches few blocks.
    uint32_t n_act_seen = gb;
    hipEvent_t te0 = nullptr, te1 = nullptr;
    if (trace) {
      SG_HIP(hipEventCreate(&te0));
      SG_HIP(hipEventCreate(&te1));
    }
    double trace_prev = 0;
    // the active list of pass p (from the flags of pass p - 1) is built by the
    // pass before it, or at a chunk end, where its count also goes to the host
    hipLaunchKernelGGL(k_active_list, dim3(1), dim3(1024), 0, st, ring[2], gb, alist, ring[0], nullptr);
    for (uint32_t pass = 0;;) {
      const uint32_t grid = 8 * ncw * ((n_act_seen + 7) / 8);
      for (uint32_t c = 0; c < chunk; c++, pass++) {
        if (pass > n + 2 + chunk) throw Error(SG_ERR_DEVICE, "relaxation did not converge");
        if (trace) SG_HIP(hipEventRecord(te0, st));
        uint32_t* changed = ring[pass % 3];
        if (c > 0)
          hipLaunchKernelGGL(k_active_list, dim3(1), dim3(1024), 0, st, ring[(pass + 2) % 3], gb, alist, changed,
                             nullptr);
        {
          TimedLaunch tl(ctx, "relax", 0.0);
          if constexpr (SPL == 2) {
            if (work)
              hipLaunchKernelGGL((k_relax_w2<B, NPW, STG / 64, GR, FRONT, true>), dim3(grid * nseg),
                                 dim3(RELAX_THREADS), 0, st, net->in_off, net->in_rec, D, n, alist, changed, stamp,
                                 pass, work, nseg);
            else
              hipLaunchKernelGGL((k_relax_w2<B, NPW, STG / 64, GR, FRONT, false>), dim3(grid * nseg),
                                 dim3(RELAX_THREADS), 0, st, net->in_off, net->in_rec, D, n, alist, changed, stamp,
                                 pass, work, nseg);
          } else {
            if (work)
              hipLaunchKernelGGL((k_relax_w<B, NPW, STG / 64, GR, FRONT, true>), dim3(grid), dim3(RELAX_THREADS), 0,
                                 st, net->in_off, net->in_rec, D, n, alist, changed, stamp, pass, work);
            else
              hipLaunchKernelGGL((k_relax_w<B, NPW, STG / 64, GR, FRONT, false>), dim3(grid), dim3(RELAX_THREADS), 0,
                                 st, net->in_off, net->in_rec, D, n, alist, changed, stamp, pass, work);
          }
        }
        SG_CHECK_LAUNCH();
        if (trace) {
          SG_HIP(hipEventRecord(te1, st));
          SG_HIP(hipEventSynchronize(te1));
          float ms = 0;
          SG_HIP(hipEventElapsedTime(&ms, te0, te1));
          unsigned long long w[WORK_SHARDS] = {};
          if (work) copy_to_host(ctx, w, work, sizeof(w));
          double tot = 0;
          for (int k = 0; k < WORK_SHARDS; k++) tot += (double)w[k];
          uint32_t na = 0;
          copy_to_host(ctx, &na, alist, 4);
          fprintf(stderr, "[apsp] group %u pass %u: %.3f ms, %u active batches, %.3f G lane-relaxations\n", g0, pass,
                  ms, na, (tot - trace_prev) / 1e9);
          trace_prev = tot;
        }
      }
      // active list of the next pass (= batches changed in the last one), its count to the host
      hipLaunchKernelGGL(k_active_list, dim3(1), dim3(1024), 0, st, ring[(pass + 2) % 3], gb, alist,
                         ring[pass % 3], ctx->apsp_ret);
      SG_CHECK_LAUNCH();
      SG_HIP(hipStreamSynchronize(st));
      n_act_seen = *(volatile uint32_t*)ctx->apsp_ret;
      if (n_act_seen == 0) break;
    }
    if (trace) {
      SG_HIP(hipEventDestroy(te0));
      SG_HIP(hipEventDestroy(te1));
    }
    SG_HIP(hipMemsetAsync(sat, 0, gb * 4ull, st));
    {
      TimedLaunch tl(ctx, "out", 12.0 * std::min<uint32_t>(gb * B, row_end - first_row) * n_used);
      const bool vec = n_used % 4 == 0 && ((uintptr_t)out_lat & 15) == 0 && ((uintptr_t)out_loss & 15) == 0;
      const uint32_t tpb = out_tpb;
      const dim3 og((n_used + 64 * tpb - 1) / (64 * tpb), gb);
#define SG_OUT(V_, T_)                                                                                          \
  hipLaunchKernelGGL((k_out_batch<B, V_, T_>), og, dim3(256), 0, st, D, n, d_used, n_used, first_row, row_end, \
                     row_begin, net->self_edge, net->e_lat, net->e_loss, out_lat, out_loss, sat)
      // (the grid above is sized for tpb: every branch launches TPB = tpb)
      if (vec && tpb == 4) SG_OUT(true, 4);
      else if (vec && tpb == 2) SG_OUT(true, 2);
      else if (vec) SG_OUT(true, 1);
      else if (tpb == 4) SG_OUT(false, 4);
      else if (tpb == 2) SG_OUT(false, 2);
      else SG_OUT(false, 1);
#undef SG_OUT
    }
    SG_CHECK_LAUNCH();
    copy_to_host(ctx, h_sat.data(), sat, gb * 4ull);
    for (uint32_t b = 0; b < gb; b++)
      if (h_sat[b])
        for (uint32_t r = 0; r < B; r++) {
          uint32_t row = first_row + b * B + r;
          if (row < row_end) wide_rows.push_back(row);
        }
  }
  if (work) {  // relaxations actually performed (relaxed arcs x lanes), for the roofline
    unsigned long long w[WORK_SHARDS];
    copy_to_host(ctx, w, work, sizeof(w));
    double total = 0;
    for (int k = 0; k < WORK_SHARDS; k++) total += (double)w[k];
    timer_add_work(ctx, "relax", total);
  }
  if (!wide_rows.empty()) run_wide(ctx, net, d_used, n_used, wide_rows, row_begin, out_lat, out_loss);
}

// A/B measurement knobs: SG_APSP_FRONTIER=0 relaxes every arc every pass;
// SG_APSP_B sources per batch (32 | 64); SG_APSP_NPW nodes per wave item;
// SG_APSP_STAGE arcs staged per wave step; SG_APSP_GROUP row reads in flight.
// Per-source LDS-resident search (sg_sssp.hip) for sparse graphs that fit a CU's
// LDS.  Bucket width: SG_APSP_DELTA (ns), else one bucket (chaotic relaxation
// over the asynchronous queue): at C3 it measured fastest (5.10 ms against
// 5.6 ms at 100 ms buckets and 6.2 ms at 50 ms), for 2.5x Dijkstra's
// relaxations against 1.06x at 50 ms -- the search is bound by its critical
// path, not by its relaxation count.
// Phases and bounds for the LDS search (sg_sssp.hip "Bounds", sg_plan.hip): phase
// 0 runs from infinity, a row of phase p >= 1 starts from bounds (and exact seeds)
// taken from neighbour rows of earlier phases; each phase is one launch, so a
// kernel boundary publishes the rows the next phase reads.  The plan is built on
// the device for every build (sg_plan.hip), so a one-shot build pays it.
// The build's end: the flagged rows' count and the self-loop check in one kernel,
// one synchronisation; the flags themselves are copied only when some row was
// flagged.  Returns the rows (absolute) that need the wide kernel.
static std::vector<uint32_t> finish_rows(sg_ctx* ctx, const uint32_t* sat, uint32_t row_begin, uint32_t rows) {
  hipStream_t st = ctx->stream;
  hipLaunchKernelGGL(k_build_finish, dim3(1), dim3(1024), 0, st, sat, rows, ctx->self_used, ctx->self_n,
                     ctx->self_cnt, ctx->apsp_ret);
  SG_CHECK_LAUNCH();
  SG_HIP(hipStreamSynchronize(st));
  const volatile uint32_t* ret = ctx->apsp_ret;
  const uint32_t n_flag = ret[4];
  if (ctx->self_used) {
    ctx->self_first = *(const volatile unsigned long long*)(ret + 2);
    ctx->self_done = true;
  }
  std::vector<uint32_t> wide_rows;
  if (n_flag) {
    std::vector<uint32_t> h_sat(rows);
    copy_to_host(ctx, h_sat.data(), sat, rows * 4ull);
    for (uint32_t r = 0; r < rows; r++)
      if (h_sat[r]) wide_rows.push_back(row_begin + r);
  }
  return wide_rows;
}

// Dense graphs (sg_dense.hip): one register-resident search per row, no plan.
static void shortest_paths_dense(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used,
                                 uint32_t row_begin, uint32_t row_end, uint64_t* out_lat, float* out_loss) {
  const uint32_t rows = row_end - row_begin;
  // (no fill: the dense kernels write every row's flag, sg_dense.hip dense_write_row)
  uint32_t* sat = ctx->r_flags.get<uint32_t>(std::max(rows, 1u));
  unsigned long long* work = ctx->count_work ? ctx->r_work.get<unsigned long long>(WORK_SHARDS) : nullptr;
  if (work) SG_HIP(hipMemsetAsync(work, 0, WORK_SHARDS * 8, ctx->stream));
  launch_sssp_dense(ctx, net, d_used, n_used, row_begin, row_end, out_lat, out_loss, sat, work);
  std::vector<uint32_t> wide_rows = finish_rows(ctx, sat, row_begin, rows);
  if (work) {
    unsigned long long w[WORK_SHARDS];
    copy_to_host(ctx, w, work, sizeof(w));
    double total = 0;
    for (int k = 0; k < WORK_SHARDS; k++) total += (double)w[k];
    timer_add_work(ctx, "sssp_dense", total);
  }
  if (!wide_rows.empty()) run_wide(ctx, net, d_used, n_used, wide_rows, row_begin, out_lat, out_loss);
}

// Sparse graphs past the LDS search (sg_bucket.hip): one delta-stepping search per row, the
// band of each bucket in LDS, later buckets in a per-workgroup arena; no plan.
static void shortest_paths_bucket(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used,
                                  uint32_t row_begin, uint32_t row_end, uint64_t* out_lat, float* out_loss) {
  const uint32_t rows = row_end - row_begin;
  uint32_t* sat = ctx->r_flags.get<uint32_t>(std::max(rows, 1u));
  SG_HIP(hipMemsetAsync(sat, 0, std::max(rows, 1u) * 4ull, ctx->stream));
  unsigned long long* work = ctx->count_work ? ctx->r_work.get<unsigned long long>(WORK_SHARDS + 16) : nullptr;
  unsigned long long* diag = work ? work + WORK_SHARDS : nullptr;
  if (work) SG_HIP(hipMemsetAsync(work, 0, (WORK_SHARDS + 16) * 8, ctx->stream));
  {
    TimedLaunch tl(ctx, "sssp_bucket", 0.0);
    launch_sssp_bucket(ctx, net, d_used, n_used, row_begin, row_end, out_lat, out_loss, sat, work, diag);
  }
  std::vector<uint32_t> wide_rows = finish_rows(ctx, sat, row_begin, rows);
  if (work) {
    unsigned long long w[WORK_SHARDS + 16];
    copy_to_host(ctx, w, work, sizeof(w));
    double total = 0;
    for (int k = 0; k < WORK_SHARDS; k++) total += (double)w[k];
    timer_add_work(ctx, "sssp_bucket", total);
    timer_add_work(ctx, "sssp_bucket_entries", (double)w[WORK_SHARDS + 1]);  // entries through the arena
    if (env_int("SG_BUCKET_DIAG", 0)) {
      const unsigned long long* d = w + WORK_SHARDS;
      const double nb = std::max(1.0, (double)d[0]);
      fprintf(stderr, "[bucket] %u rows: %.1f buckets, %.0f entries, %.2f far steps, %.0f pops in %.0f claims, "
              "%.0f relaxations (%.3f x arcs) per row\n", rows, d[0] / (double)rows, d[1] / (double)rows,
              d[2] / (double)rows, d[3] / (double)rows, d[8] / (double)rows, total / rows,
              total / rows / std::max(1u, net->n_arcs));
      fprintf(stderr, "[bucket] cycles per bucket (thread 0): phase 0 %.0f, phase 1 %.0f, phase 2 %.0f; output per row %.0f\n",
              d[4] / nb, d[5] / nb, d[6] / nb, d[7] / (double)rows);
      fprintf(stderr, "[bucket] band kernel, wave 0 per bucket: offsets %.0f, arcs (with appends) %.0f, appends %.0f, store wait %.0f; "
              "band splits per row %.2f\n", d[9] / nb, d[10] / nb, d[11] / nb, d[12] / nb, d[15] / (double)rows);
      fprintf(stderr, "[bucket] band kernel, thread 0 per bucket in the load step: entry loads %.0f, hash %.0f, barrier wait %.0f\n",
              d[8] / nb, d[13] / nb, d[14] / nb);
      const double ncl = std::max(1.0, (double)d[8]);
      fprintf(stderr, "[bucket] per wave and bucket: load step %.0f cyc, idle %.0f; per claim: to offsets %.0f, to "
              "arcs %.0f (sum over arc rounds), appends %.0f, claim total %.0f\n", d[9] / nb / 4, d[14] / nb / 4,
              d[10] / ncl, d[11] / ncl, d[12] / ncl, d[13] / ncl);
    }
  }
  if (!wide_rows.empty()) run_wide(ctx, net, d_used, n_used, wide_rows, row_begin, out_lat, out_loss);
}

static void shortest_paths_lds(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used, uint32_t row_begin, uint32_t row_end, uint64_t* out_lat,
                               float* out_loss) {
  hipStream_t st = ctx->stream;
  const uint32_t rows = row_end - row_begin;
  uint32_t* sat = ctx->r_flags.get<uint32_t>(rows);  // zeroed by the plan's first kernel, else here
  unsigned long long* work = ctx->count_work ? ctx->r_work.get<unsigned long long>(WORK_SHARDS) : nullptr;
  if (work) SG_HIP(hipMemsetAsync(work, 0, WORK_SHARDS * 8, st));
  const char* ds = getenv("SG_APSP_DELTA");
  double dd = ds && *ds ? atof(ds) : 4294967295.0;
  const uint32_t delta = (uint32_t)std::min(4294967295.0, std::max(1.0, dd));
  // SG_SSSP_DIAG=1 (with counting timers): per-row cycle and phase statistics on stderr
  const bool diag_on = work && env_int("SG_SSSP_DIAG", 0) != 0;
  const uint32_t n_diag = std::min<uint32_t>(rows, 4096);
  unsigned long long* diag = diag_on ? ctx->r_misc.get<unsigned long long>((size_t)n_diag * 8) : nullptr;
  if (diag) SG_HIP(hipMemsetAsync(diag, 0, (size_t)n_diag * 64, st));
  // Phases (sg_plan.hip) from 8 rows per CU: with fewer, the phase boundaries cost
  // more than the bounds save (tools/sssp_ab.py, C3 graph: 1,250 rows 0.78 against
  // 0.76 ms unbounded, a 2,000-node build 0.45 against 0.43; 2,500 rows 1.30
  // against 1.38, a 4,000-node build 0.97 against 1.07).  SG_SSSP_SEEDS=0 never, =2 always.
  const int seeds_env = env_int("SG_SSSP_SEEDS", 1);
  // Flagged rows (sg_sssp.hip): the plan's rows in ONE launch, in phase order, each row
  // taking the bound rows already published when it starts -- no phase boundaries, so the
  // bounds pay even with few rows per CU.  The default for a row block (a rank's share of a
  // sharded build, or a RoutingInfo fill block); the whole table keeps the phased launches,
  // which it builds as fast (one box, tools/sssp_ab.py, C3 graph, tables bit-identical:
  // 10k rows 3.187 against 3.185 ms; row blocks of 5,000 1.93 against 1.99, 2,500 1.13
  // against 1.20, 1,250 0.685 against 0.706).  SG_SSSP_FLAGGED=0 / 1 forces it.
  // Below 6 rows per CU neither pays: the plan and the seeding cost more than the bounds save
  // (r7i-r7j, C3 graph, the hybrid lane path, tables identical: 640 rows 0.351 ms unbounded against
  // 0.398 flagged, 1,250 rows 0.558 against 0.581; 2,500 rows 1.044 against 0.948 flagged)
  const int flag_env = env_int("SG_SSSP_FLAGGED", -1);
  const bool few_rows = rows < 6u * (uint32_t)std::max(1, ctx->n_cu);
  const bool flagged = seeds_env != 0 && (flag_env == 1 || (flag_env < 0 && rows < n_used && !few_rows));
  const bool phased = !flagged && seeds_env != 0 && (seeds_env == 2 || rows >= 8u * (uint32_t)ctx->n_cu);
  // without a plan: the row flags and the persistent workgroups' claim counters zeroed by one
  // launch (two fills cost two dispatches and ~10 us of host time in a one-shot block build)
  uint32_t* claim_ctr = nullptr;
  if (!phased && !flagged) {
    claim_ctr = ctx->r_items.get<uint32_t>(2);
    hipLaunchKernelGGL(k_zero2, dim3(grid_for((size_t)rows + 2, 256, 1024)), dim3(256), 0, st, sat, rows,
                       claim_ctr, 2u);
    SG_CHECK_LAUNCH();
  }
  if (flagged) {
    const uint32_t per_cu = rows / std::max(1, ctx->n_cu);
    const int n_phase = std::max(2, std::min(SSSP_PHASES_MAX, env_int("SG_SSSP_PHASES", per_cu >= 16 ? 3 : 2)));
    const int kb = std::max(1, std::min(SSSP_KB_MAX, env_int("SG_SSSP_BOUNDS", 2)));
    const bool exact = env_int("SG_SSSP_EXACT", 1) != 0 && n_used == net->n_nodes;
    const int hops = std::max(1, std::min(env_int("SG_SSSP_HOPS", 3), 3));
    uint32_t* done = ctx->r_done.get<uint32_t>(std::max(rows, 1u));
    const SsspDevPlan plan =
        sssp_device_plan(ctx, net, d_used, n_used, row_begin, row_end, n_phase, kb, exact, hops, 0u, sat, done);
    TimedLaunch tl(ctx, "sssp", 0.0);
    launch_sssp_lds(ctx, net->out_off, net->out_arc, net->n_nodes, net->n_arcs, d_used, n_used, row_begin, row_end,
                    net->self_edge, net->e_lat, net->e_loss, out_lat, out_loss, sat, delta, work, diag, plan.list, rows,
                    plan.ub_row, plan.ub_w, nullptr, 0, plan.ctr, done);
  } else if (phased) {
    // phases by rows per CU (one box, tools/sssp_ab.py --rows, C3 graph): 39 rows per CU
    // (10k rows) 4 phases; 19.5 (a half) 3 phases, 2.25 against 2.57 ms unbounded;
    // 9.8 (a quarter) 2 phases, 1.30 against 1.38 ms
    const uint32_t per_cu = rows / std::max(1, ctx->n_cu);
    const int n_phase = std::max(2, std::min(SSSP_PHASES_MAX,
                                             env_int("SG_SSSP_PHASES", per_cu >= 16 ? 3 : 2)));
    const int kb = std::max(1, std::min(SSSP_KB_MAX, env_int("SG_SSSP_BOUNDS", 2)));
    // exact seeds need a column for every node (see sg_sssp.hip "Exact seeds")
    const bool exact = env_int("SG_SSSP_EXACT", 1) != 0 && n_used == net->n_nodes;
    const int hops = std::max(1, std::min(env_int("SG_SSSP_HOPS", 3), 3));
    // Landmarks (sg_plan.hip header; undirected graphs): SG_SSSP_LANDMARKS rows first, the
    // rest of phase 0 bounded through them.  Off by default: at C3 (tools/sssp_ab.py, one
    // box, tables bit-identical) 256 landmarks cut phase 0 from 1.30 to 0.36 ms but the
    // landmark-bounded rows took 113 us each against 129 unbounded and 66 for rows bounded
    // by a neighbour: the build took 3.53 ms against 3.43 (128: 3.54, 512: 3.67).
    const int land_env = env_int("SG_SSSP_LANDMARKS", 0);
    const uint32_t n_land = net->directed || land_env <= 0 ? 0u : (uint32_t)land_env;
    const SsspDevPlan plan =
        sssp_device_plan(ctx, net, d_used, n_used, row_begin, row_end, n_phase, kb, exact, hops, n_land, sat);
    if (const int warm = env_int("SG_PLAN_WARM", 0))
      hipLaunchKernelGGL(k_busy, dim3(4 * ctx->n_cu), dim3(256), 0, ctx->stream, (uint32_t)warm, (float*)nullptr);
    // SG_PLAN_SYNC=1 (A/B diagnostics): read the phase sizes to the host and launch with host-known counts
    std::vector<uint32_t> hctl;
    if (env_int("SG_PLAN_SYNC", 0)) {
      hctl.resize(2 * SSSP_PHASES_MAX);
      copy_to_host(ctx, hctl.data(), plan.ctl, hctl.size() * 4);
    }
    for (int ph = 0; ph < plan.n_phase; ph++) {
      const bool bounded = ph > 0;
      TimedLaunch tl(ctx, bounded ? "sssp_bounded" : "sssp", 0.0);
      if (!hctl.empty()) {
        const uint32_t b0 = hctl[2 * ph], cnt = hctl[2 * ph + 1];
        launch_sssp_lds(ctx, net->out_off, net->out_arc, net->n_nodes, net->n_arcs, d_used, n_used, row_begin,
                        row_end, net->self_edge, net->e_lat, net->e_loss, out_lat, out_loss, sat, delta, work,
                        ph + 1 == plan.n_phase ? diag : nullptr, plan.list + b0, cnt,
                        bounded ? plan.ub_row + (size_t)b0 * SSSP_KB_MAX : nullptr,
                        bounded ? plan.ub_w + (size_t)b0 * SSSP_KB_MAX : nullptr);
        if (ph == 0 && plan.landmarks) sssp_landmark_bounds(ctx, plan, n_used, row_begin, out_lat, sat, kb);
        continue;
      }
      launch_sssp_lds(ctx, net->out_off, net->out_arc, net->n_nodes, net->n_arcs, d_used, n_used, row_begin,
                      row_end, net->self_edge, net->e_lat, net->e_loss, out_lat, out_loss, sat, delta, work,
                      ph + 1 == plan.n_phase ? diag : nullptr, plan.list, rows, bounded ? plan.ub_row : nullptr,
                      bounded ? plan.ub_w : nullptr, plan.ctl, ph, plan.ctr + 2 * ph);
      if (ph == 0 && plan.landmarks) sssp_landmark_bounds(ctx, plan, n_used, row_begin, out_lat, sat, kb);
    }
  } else {
    TimedLaunch tl(ctx, "sssp", 0.0);
    launch_sssp_lds(ctx, net->out_off, net->out_arc, net->n_nodes, net->n_arcs, d_used, n_used, row_begin,
                    row_end, net->self_edge, net->e_lat, net->e_loss, out_lat, out_loss, sat, delta, work, diag,
                    nullptr, 0, nullptr, nullptr, nullptr, 0, claim_ctr);
  }
  if (diag) {
    std::vector<unsigned long long> h((size_t)n_diag * 8);
    copy_to_host(ctx, h.data(), diag, h.size() * 8);
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    double setup = 0;
    for (uint32_t r = 0; r < n_diag; r++) {
      for (int k = 0; k < 8; k++) a[k] += (double)h[(size_t)r * 8 + k];
      setup += (double)(h[(size_t)r * 8 + 3] >> 24);
      a[3] -= (double)(h[(size_t)r * 8 + 3] >> 24 << 24);
    }
    fprintf(stderr, "[sssp] mean setup (init + bound rows) %.0f cyc of the search\n", setup / n_diag);
    fprintf(stderr, "[sssp] per-wave cycles summed over a row's 16 waves: claim+wait %.0f, pop %.0f, steps %.0f "
            "(per pop: %.0f, %.0f)\n", a[5] / n_diag, a[6] / n_diag, a[7] / n_diag, a[6] / std::max(1.0, a[2]),
            a[7] / std::max(1.0, a[2]));
    fprintf(stderr, "[sssp] delta %u ns, %u rows: mean search %.0f cyc, output %.0f cyc, %.1f wave pops, %.1f buckets, "
            "%.0f relaxations (%.2f x arcs)\n", delta, n_diag, a[0] / n_diag, a[1] / n_diag, a[2] / n_diag,
            a[3] / n_diag, a[4] / n_diag, a[4] / n_diag / std::max(1u, net->n_arcs));
  }
  std::vector<uint32_t> wide_rows = finish_rows(ctx, sat, row_begin, rows);
  if (work) {
    unsigned long long w[WORK_SHARDS];
    copy_to_host(ctx, w, work, sizeof(w));
    double total = 0;
    for (int k = 0; k < WORK_SHARDS; k++) total += (double)w[k];
    timer_add_work(ctx, "sssp", total);
  }
  if (!wide_rows.empty()) run_wide(ctx, net, d_used, n_used, wide_rows, row_begin, out_lat, out_loss);
}

static void shortest_paths(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, const uint32_t* h_used,
                           uint32_t n_used, uint32_t row_begin, uint32_t row_end, uint64_t* out_lat,
                           float* out_loss) {
  // (Round 3 also built a team search for graphs past one CU's LDS, K workgroups per
  // row: 1.5x Dijkstra's relaxations at C5 but 646 ms against the slab's 249 ms, so
  // it was removed in round 4; DESIGN.md, "Team search".)
  // SG_APSP_LDS=0 forces the batched-source slab kernel.  The LDS search takes
  // sparse graphs (mean out-degree <= 64); on dense ones the slab kernel shares
  // each arc record among 64 sources (C2, 1,200-node complete graph: 3.6 ms
  // against 6.8-9.2 ms for the LDS search).
  const bool sparse = net->n_nodes && net->n_arcs <= 64ull * net->n_nodes;
  // Dense graphs up to DENSE_MAX nodes (C2): the register-resident search of sg_dense.hip,
  // Dijkstra's n^2 relaxations per row (SG_APSP_DENSE=0 or SG_APSP_LDS=0: the slab kernel).
  if (env_int("SG_APSP_LDS", 1) != 0 && env_int("SG_APSP_DENSE", 1) != 0 && !sparse &&
      sssp_dense_fits(net->n_nodes)) {
    shortest_paths_dense(ctx, net, d_used, n_used, row_begin, row_end, out_lat, out_loss);
    return;
  }
  // SG_APSP_BUCKET: 1 forces the bucketed search on any sparse graph (tests), 0 keeps the slab
  // kernel past the LDS search
  const int bucket_env = env_int("SG_APSP_BUCKET", -1);
  const bool arcs_ok = (uint64_t)net->n_arcs * 12 < (1ull << 31);
  if (env_int("SG_APSP_LDS", 1) != 0 && sparse && arcs_ok && bucket_env != 0 && sssp_bucket_fits(net->n_nodes) &&
      (bucket_env == 1 || !sssp_lds_fits(net->n_nodes))) {
    shortest_paths_bucket(ctx, net, d_used, n_used, row_begin, row_end, out_lat, out_loss);
    return;
  }
  if (env_int("SG_APSP_LDS", 1) != 0 && sparse && sssp_lds_fits(net->n_nodes) && arcs_ok) {
    shortest_paths_lds(ctx, net, d_used, n_used, row_begin, row_end, out_lat, out_loss);
    return;
  }
  const bool front = env_int("SG_APSP_FRONTIER", 1) != 0;
  // dense graphs (more than ~600 in-arcs per node: C2's complete graph) relax
  // faster in 32-source batches with arc segments (3.49 vs 3.66 ms at C2)
  const bool dense = net->n_nodes && (double)net->n_arcs / net->n_nodes > 600.0;
  const int bsz = env_int("SG_APSP_B", dense ? 32 : 64);
  const int spl = env_int("SG_APSP_SPL", 2);  // sources per lane: 2 = k_relax_w2 (the default)
  // defaults: the fastest measured configuration of each kernel (tools/apsp_variants.py)
  const int npw = env_int("SG_APSP_NPW", spl == 2 ? 4 : 8), stg = env_int("SG_APSP_STAGE", spl == 2 ? 64 : 128);
  const int gr = env_int("SG_APSP_GROUP", spl == 2 ? 3 : 8);
  if (spl == 2) {
#define SG_SP2(B_, NPW_, STG_, GR_)                                                                      \
  if (bsz == B_ && npw == NPW_ && stg == STG_ && gr == GR_) {                                           \
    if (front)                                                                                          \
      shortest_paths_t<B_, NPW_, STG_, GR_, true, 2>(ctx, net, d_used, n_used, row_begin, row_end, out_lat, \
                                                     out_loss);                                         \
    else                                                                                                \
      shortest_paths_t<B_, NPW_, STG_, GR_, false, 2>(ctx, net, d_used, n_used, row_begin, row_end,      \
                                                      out_lat, out_loss);                               \
    return;                                                                                             \
  }
    SG_SP2(64, 8, 128, 8)
    SG_SP2(64, 8, 128, 4)
    SG_SP2(64, 8, 128, 2)
    SG_SP2(64, 8, 128, 6)
    SG_SP2(64, 8, 64, 4)
    SG_SP2(64, 4, 64, 4)
    SG_SP2(64, 4, 128, 4)
    SG_SP2(64, 2, 64, 4)
    SG_SP2(64, 4, 64, 3)
    SG_SP2(64, 4, 64, 5)
    SG_SP2(64, 16, 128, 4)
    SG_SP2(32, 4, 64, 3)
    SG_SP2(32, 4, 64, 2)
    SG_SP2(32, 8, 64, 3)
    SG_SP2(32, 8, 128, 3)
    SG_SP2(32, 4, 128, 3)
#undef SG_SP2
    throw Error(SG_ERR_INVALID_ARG, "unsupported SG_APSP_SPL=2 configuration");
  }
#define SG_SP(B_, NPW_, STG_, GR_)                                                                       \
  if (bsz == B_ && npw == NPW_ && stg == STG_ && gr == GR_) {                                           \
    if (front)                                                                                          \
      shortest_paths_t<B_, NPW_, STG_, GR_, true>(ctx, net, d_used, n_used, row_begin, row_end, out_lat,  \
                                                  out_loss);                                            \
    else                                                                                                \
      shortest_paths_t<B_, NPW_, STG_, GR_, false>(ctx, net, d_used, n_used, row_begin, row_end, out_lat, \
                                                   out_loss);                                           \
    return;                                                                                             \
  }
  SG_SP(64, 8, 128, 8)
  SG_SP(64, 8, 128, 16)
  SG_SP(64, 16, 128, 8)
  SG_SP(64, 4, 64, 8)
  SG_SP(32, 8, 128, 8)
  SG_SP(32, 16, 128, 8)
#undef SG_SP
  throw Error(SG_ERR_INVALID_ARG, "unsupported SG_APSP_B / SG_APSP_NPW / SG_APSP_STAGE / SG_APSP_GROUP");
}

static void direct_paths(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, const uint32_t* h_used,
                         uint32_t n_used, uint32_t row_begin, uint32_t row_end, uint64_t* out_lat,
                         float* out_loss) {
  hipStream_t st = ctx->stream;
  const uint32_t n = net->n_nodes;
  std::vector<uint32_t> map(n, ~0u);
  for (uint32_t j = 0; j < n_used; j++) map[h_used[j]] = j;
  uint32_t* d_map = ctx->r_map.get<uint32_t>(n);
  SG_HIP(hipMemcpyAsync(d_map, map.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
  size_t count = (size_t)(row_end - row_begin) * n_used;
  uint32_t* cnt = ctx->r_pair_cnt.get<uint32_t>(count);
  uint32_t* edge = ctx->r_pair_edge.get<uint32_t>(count);
  SG_HIP(hipMemsetAsync(cnt, 0, count * 4, st));
  if (net->n_edges)
    hipLaunchKernelGGL(k_pair_count, dim3(grid_for(net->n_edges, 256, 8192)), dim3(256), 0, st,
                       net->e_src, net->e_dst, net->n_edges, (int)net->directed, d_map, n_used,
                       row_begin, row_end, cnt, edge);
  unsigned long long* first = ctx->r_err.get<unsigned long long>(4);
  SG_HIP(hipMemsetAsync(first, 0xff, 8, st));
  hipLaunchKernelGGL(k_pair_out, dim3(grid_for(count, 256, 65536)), dim3(256), 0, st, cnt, edge,
                     count, n_used, row_begin, net->e_lat, net->e_loss, out_lat, out_loss, first);
  SG_CHECK_LAUNCH();
  unsigned long long h = 0;
  copy_to_host(ctx, &h, first, 8);
  if (h != ~0ull) {
    unsigned long long lin = h >> 1;
    uint32_t i = (uint32_t)(lin / n_used), j = (uint32_t)(lin % n_used);
    std::string a = node_name(net, h_used[i]), b = node_name(net, h_used[j]);
    if (h & 1) throw Error(SG_ERR_MULTI_EDGE, "More than one edge connecting node " + a + " to " + b, i, j);
    throw Error(SG_ERR_NO_EDGE, "No edge connecting node " + a + " to " + b, i, j);
  }
}

}  // namespace sg

extern "C" {

int32_t sg_net_create(sg_ctx* ctx, const sg_graph* g, sg_net** out) {
  if (!g || !out) return SG_ERR_INVALID_ARG;
  *out = nullptr;
  sg_net* net = nullptr;
  int32_t rc = sg::guarded(ctx, [&] {
    net = new sg_net();
    net->serial = ++ctx->net_serial;
    sg::build_net(ctx, g, net);
  });
  if (rc != SG_OK) {
    delete net;
    return rc;
  }
  *out = net;
  return SG_OK;
}

void sg_net_destroy(sg_net* net) {
  if (!net) return;
  sg_ctx* ctx = net->ctx;
  if (ctx) {
    (void)hipSetDevice(ctx->device);
    hipEvent_t ev = nullptr;
    if (net->mem && hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess &&
        hipEventRecord(ev, ctx->stream) == hipSuccess) {
      ctx->net_pool.push_back({net->mem, net->mem_bytes, ev});
      net->mem = nullptr;
      while (ctx->net_pool.size() > 4) {  // keep a few blocks; release the oldest
        auto& old = ctx->net_pool.front();
        (void)hipEventSynchronize(old.freed);
        (void)hipEventDestroy(old.freed);
        (void)hipFree(old.p);
        ctx->net_pool.erase(ctx->net_pool.begin());
      }
    } else if (ev) {
      (void)hipEventDestroy(ev);
    }
  }
  delete net;
}

namespace sg {
// The used-node list: every index in range, none twice.  One branch-free pass; only a bad
// list is walked again, entry by entry, for the first bad entry's error.
static void check_node_list(const sg_net* net, const uint32_t* nodes, uint32_t n_used) {
  const uint32_t n = net->n_nodes;
  std::vector<uint8_t> seen((size_t)n + 1, 0);  // the spare last byte takes out-of-range ids
  uint32_t bad = 0;
  for (uint32_t j = 0; j < n_used; j++) {
    const uint32_t v = nodes[j];
    const uint32_t out = v >= n;
    const uint32_t x = out ? n : v;
    bad |= out | (uint32_t)seen[x];
    seen[x] = 1;
  }
  if (!bad) return;
  std::fill(seen.begin(), seen.end(), (uint8_t)0);
  for (uint32_t j = 0; j < n_used; j++) {
    if (nodes[j] >= n) throw Error(SG_ERR_INVALID_ARG, "node index out of range");
    if (seen[nodes[j]]++) throw Error(SG_ERR_INVALID_ARG, "duplicate node in node list");
  }
}
}  // namespace sg

int32_t sg_routing_build(sg_ctx* ctx, sg_net* net, const uint32_t* nodes, uint32_t n_used,
                         uint32_t row_begin, uint32_t row_end, uint32_t flags,
                         uint64_t* out_latency_ns, float* out_packet_loss) {
  return sg::guarded(ctx, [&] {
    using namespace sg;
    if (!net || net->ctx != ctx) throw Error(SG_ERR_INVALID_ARG, "network belongs to another context");
    if (row_begin > row_end || row_end > n_used) throw Error(SG_ERR_INVALID_ARG, "bad row range");
    if (n_used && !nodes) throw Error(SG_ERR_INVALID_ARG, "null node list");
    if (row_end > row_begin && (!out_latency_ns || !out_packet_loss))
      throw Error(SG_ERR_INVALID_ARG, "null output");
    check_node_list(net, nodes, n_used);
    if (n_used == 0) return;
    hipStream_t st = ctx->stream;
    uint32_t* d_used = ctx->r_used.get<uint32_t>(n_used);
    {
      char* hu = stage_acquire(ctx, 1, (size_t)n_used * 4);
      memcpy(hu, nodes, (size_t)n_used * 4);
      SG_HIP(hipMemcpyAsync(d_used, hu, (size_t)n_used * 4, hipMemcpyHostToDevice, st));
      stage_release(ctx, 1);
    }
    const bool shortest = flags & SG_ROUTE_SHORTEST_PATH;
    // The reference checks every used node's self-loop (graph/mod.rs:211-217),
    // whichever rows this call computes.
    if (row_end == row_begin) {
      if (shortest) raise_self_loops(ctx, net, launch_self_loops(ctx, net, d_used, n_used), nodes);
      return;
    }
    const size_t count = (size_t)(row_end - row_begin) * n_used;
    const bool dev_out = flags & SG_ROUTE_OUT_DEVICE;
    uint64_t* o_lat = dev_out ? out_latency_ns : ctx->r_out_lat.get<uint64_t>(count);
    float* o_loss = dev_out ? out_packet_loss : ctx->r_out_loss.get<float>(count);
    if (shortest) {
      // the check of every used node's self-loop (graph/mod.rs:210-217) rides on the LDS
      // search's final kernel (k_build_finish); the other kernels leave it to a launch of its own
      ctx->self_used = d_used;
      ctx->self_n = n_used;
      ctx->self_cnt = net->self_cnt;
      ctx->self_done = false;
      struct Clear {  // however the build ends, no later kernel reads this net's arrays for the check
        sg_ctx* c;
        ~Clear() {
          c->self_used = nullptr;
          c->self_cnt = nullptr;
          c->self_done = false;
        }
      } clear{ctx};
      try {
        shortest_paths(ctx, net, d_used, nodes, n_used, row_begin, row_end, o_lat, o_loss);
      } catch (const Error&) {
        ctx->self_done = false;  // (the search may have failed before its final kernel)
        raise_self_check(ctx, net, d_used, n_used, nodes);  // a self-loop error first (graph/mod.rs:210-219)
        throw;
      }
      raise_self_check(ctx, net, d_used, n_used, nodes);
    } else
      direct_paths(ctx, net, d_used, nodes, n_used, row_begin, row_end, o_lat, o_loss);
    if (!dev_out) {
      SG_HIP(hipMemcpyAsync(out_latency_ns, o_lat, count * 8, hipMemcpyDeviceToHost, st));
      SG_HIP(hipMemcpyAsync(out_packet_loss, o_loss, count * 4, hipMemcpyDeviceToHost, st));
    }
    SG_HIP(hipStreamSynchronize(st));
  });
}

// The whole table into a host RoutingInfo (sg_route_info.hip): row blocks are
// built into one of two device staging buffers, packed into 8-byte cells and
// copied to the object's pinned host array on a second stream while the next
// block builds.  The copy (8 bytes per cell over PCIe) is what binds.
int32_t sg_routing_info_fill(sg_ctx* ctx, sg_net* net, const uint32_t* nodes, uint32_t flags, sg_routing_info* ri) {
  return sg::guarded(ctx, [&] {
    using namespace sg;
    if (!net || net->ctx != ctx) throw Error(SG_ERR_INVALID_ARG, "network belongs to another context");
    if (!ri) throw Error(SG_ERR_INVALID_ARG, "null routing info");
    const uint32_t n_used = ri->n;
    if (n_used && !nodes) throw Error(SG_ERR_INVALID_ARG, "null node list");
    check_node_list(net, nodes, n_used);
    ri->filled = false;
    ri->min_lat = UINT64_MAX;
    ri->wide.clear();
    std::fill(ri->row_set.begin(), ri->row_set.end(), 0);
    ri->rows_set = 0;
    if (n_used == 0) {
      ri->filled = true;
      return;
    }
    hipStream_t st = ctx->stream;
    if (!ctx->copy_stream) {
      SG_HIP(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
      for (int b = 0; b < 2; b++) {
        SG_HIP(hipEventCreateWithFlags(&ctx->stage_done[b], hipEventDisableTiming));
        SG_HIP(hipEventCreateWithFlags(&ctx->stage_copied[b], hipEventDisableTiming));
      }
    }
    // an earlier fill that failed may have left copies in flight into its staging buffers
    SG_HIP(hipStreamSynchronize(ctx->copy_stream));
    uint32_t* d_used = ctx->r_used.get<uint32_t>(n_used);
    {
      char* hu = stage_acquire(ctx, 1, (size_t)n_used * 4);
      memcpy(hu, nodes, (size_t)n_used * 4);
      SG_HIP(hipMemcpyAsync(d_used, hu, (size_t)n_used * 4, hipMemcpyHostToDevice, st));
      stage_release(ctx, 1);
    }
    const bool shortest = flags & SG_ROUTE_SHORTEST_PATH;
    if (shortest) raise_self_loops(ctx, net, launch_self_loops(ctx, net, d_used, n_used), nodes);
    // blocks of about 1/8 of the table (at least 64 rows, whole 64-row batches)
    uint32_t rows = (uint32_t)std::max(64, env_int("SG_RI_BLOCK_ROWS", (int)((n_used + 7) / 8)));
    rows = std::min(n_used, (rows + 63) / 64 * 64);
    uint64_t* slat[2];
    float* sloss[2];
    uint64_t* spack[2];
    for (int b = 0; b < 2; b++) {
      slat[b] = ctx->r_stage_lat[b].get<uint64_t>((size_t)rows * n_used);
      sloss[b] = ctx->r_stage_loss[b].get<float>((size_t)rows * n_used);
      spack[b] = ctx->r_stage_pack[b].get<uint64_t>((size_t)rows * n_used);
    }
    const unsigned nbp = grid_for((size_t)rows * n_used / 2, 256, 4096);
    uint64_t m = UINT64_MAX;
    int k = 0;
    try {
      for (uint32_t r0 = 0; r0 < n_used; r0 += rows, k++) {
        const uint32_t r1 = std::min(n_used, r0 + rows), b = k & 1;
        ctx->in_fill = true;
        try {
          if (shortest)
            shortest_paths(ctx, net, d_used, nodes, n_used, r0, r1, slat[b], sloss[b]);
          else
            direct_paths(ctx, net, d_used, nodes, n_used, r0, r1, slat[b], sloss[b]);
        } catch (...) {
          ctx->in_fill = false;
          throw;
        }
        ctx->in_fill = false;
        const size_t cells = (size_t)(r1 - r0) * n_used;
        // (workspace fetched after the build, which may grow these buffers)
        unsigned long long* ctl = ctx->r_err.get<unsigned long long>(4);
        SG_HIP(hipMemsetAsync(ctl, 0xff, 8, st));
        SG_HIP(hipMemsetAsync(ctl + 1, 0, 8, st));
        if (k >= 2) SG_HIP(hipStreamWaitEvent(st, ctx->stage_copied[b], 0));  // block k - 2 left spack[b]
        hipLaunchKernelGGL(k_pack_cells, dim3(nbp), dim3(256), 0, st, slat[b], sloss[b], cells, spack[b], ctl);
        SG_CHECK_LAUNCH();
        SG_HIP(hipEventRecord(ctx->stage_done[b], st));
        SG_HIP(hipStreamWaitEvent(ctx->copy_stream, ctx->stage_done[b], 0));
        SG_HIP(hipMemcpyAsync(ri->cell + (size_t)r0 * n_used, spack[b], cells * 8, hipMemcpyDeviceToHost,
                              ctx->copy_stream));
        SG_HIP(hipEventRecord(ctx->stage_copied[b], ctx->copy_stream));
        unsigned long long h[2] = {0, 0};
        copy_to_host(ctx, h, ctl, 16);  // (the next block's build starts after this sync; the copy runs on)
        m = std::min<uint64_t>(m, h[0]);
        if (h[1]) {  // paths of 4.29 s or more: their u64 latencies to the side table
          uint64_t* list = ctx->r_misc.get<uint64_t>(2 * h[1]);
          SG_HIP(hipMemsetAsync(ctl + 1, 0, 8, st));
          hipLaunchKernelGGL(k_wide_list, dim3(grid_for(cells, 256, 4096)), dim3(256), 0, st, slat[b], cells,
                             (uint64_t)r0 * n_used, ctl + 1, list);
          SG_CHECK_LAUNCH();
          std::vector<uint64_t> hl(2 * h[1]);
          copy_to_host(ctx, hl.data(), list, hl.size() * 8);
          for (size_t i = 0; i < h[1]; i++) ri->wide.push_back({hl[2 * i], hl[2 * i + 1]});
        }
      }
    } catch (...) {
      (void)hipStreamSynchronize(ctx->copy_stream);  // no copy may still run into the object
      throw;
    }
    SG_HIP(hipStreamSynchronize(ctx->copy_stream));
    std::sort(ri->wide.begin(), ri->wide.end(),
              [](const sg_routing_info::Wide& x, const sg_routing_info::Wide& y) { return x.cell < y.cell; });
    std::fill(ri->row_set.begin(), ri->row_set.end(), 2);  // written; per-row minima not kept
    ri->rows_set = n_used;
    ri->min_lat = m;
    ri->filled = true;
  });
}

int32_t sg_routing_min_latency(sg_ctx* ctx, const uint64_t* d_latency_ns, size_t count,
                               uint64_t* out_min) {
  return sg::guarded(ctx, [&] {
    using namespace sg;
    if (!out_min || (count && !d_latency_ns)) throw Error(SG_ERR_INVALID_ARG, "null argument");
    unsigned long long* m = ctx->r_err.get<unsigned long long>(4);
    SG_HIP(hipMemsetAsync(m, 0xff, 8, ctx->stream));
    if (count) {
      const unsigned nb = grid_for(count, 256, 2048);
      unsigned long long* part = ctx->r_misc.get<unsigned long long>(nb);
      hipLaunchKernelGGL(k_min_u64, dim3(nb), dim3(256), 0, ctx->stream, d_latency_ns, count, part);
      hipLaunchKernelGGL(k_min_final, dim3(1), dim3(256), 0, ctx->stream, part, nb, m);
    }
    SG_CHECK_LAUNCH();
    unsigned long long h = 0;
    copy_to_host(ctx, &h, m, 8);
    *out_min = h;
  });
}

}  // extern "C"
