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
// Kernel: batched-source pull relaxation.  A wave owns one destination node v
// of one 64-source batch; lane = source.  The batch's distance slab is laid out
// [node][64 sources], so each in-arc (u -> v) costs one coalesced 512-B read of
// D[u][0..63] and 64 independent relaxations.  In-arcs are read through the
// scalar path (wave-uniform).  The key is packed: (lat << 30) | f32 bits(loss),
// so one u64 min is the lexicographic PathProperties comparison and one 64-bit
// store is an untorn (lat, loss) update -> in-place (Gauss-Seidel) passes.
// Rows whose keys saturate (latency >= 2^34-1 ns, or unreachable) are redone
// with a wide (u64 latency, f32 loss) Jacobi kernel.
#include <algorithm>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "sg_device.h"
#include "sg_internal.h"

struct sg_net {
  sg_ctx* ctx = nullptr;
  uint32_t n_nodes = 0, n_edges = 0, n_arcs = 0;
  bool directed = false;
  std::vector<uint32_t> gml_id;
  // GML edge list (device)
  uint32_t* e_src = nullptr;
  uint32_t* e_dst = nullptr;
  uint64_t* e_lat = nullptr;
  float* e_loss = nullptr;
  // in-arc CSC without self-loops (device)
  uint32_t* in_off = nullptr;  // n_nodes + 1
  uint32_t* in_src = nullptr;
  uint64_t* in_lat = nullptr;
  float* in_om = nullptr;  // 1f32 - loss
  // self-loops
  uint32_t* self_cnt = nullptr;
  uint32_t* self_edge = nullptr;
  ~sg_net() {
    void* ps[] = {e_src, e_dst, e_lat, e_loss, in_off, in_src, in_lat, in_om, self_cnt, self_edge};
    for (void* p : ps)
      if (p) (void)hipFree(p);
  }
};

namespace sg {

constexpr int BATCH = 64;         // sources per batch = wave width
constexpr int RELAX_WAVES = 4;    // waves per block
constexpr int RELAX_BLOCK = RELAX_WAVES * 64;
constexpr int WORK_SHARDS = 64;  // relaxation counter shards (measurement only)
constexpr int ARC_CHUNK = 1024;  // in-arcs staged in LDS per block step

// ---------------------------------------------------------------------------
// Graph upload: CSC of in-arcs (both directions when undirected, petgraph
// semantics graph/mod.rs:137-152), self-loop census for get_edge_weight(n, n).
// ---------------------------------------------------------------------------
__global__ void k_count_arcs(const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                             uint32_t m, int directed, uint32_t* __restrict__ indeg,
                             uint32_t* __restrict__ self_cnt, uint32_t* __restrict__ self_edge) {
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < m; e += gridDim.x * blockDim.x) {
    uint32_t s = src[e], d = dst[e];
    if (s == d) {
      atomicAdd(&self_cnt[s], 1u);
      self_edge[s] = e;  // meaningful only when the count ends at 1
    } else {
      atomicAdd(&indeg[d], 1u);
      if (!directed) atomicAdd(&indeg[s], 1u);
    }
  }
}

__global__ void k_scatter_arcs(const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                               const uint64_t* __restrict__ lat, const float* __restrict__ loss,
                               uint32_t m, int directed, uint32_t* __restrict__ cursor,
                               uint32_t* __restrict__ in_src, uint64_t* __restrict__ in_lat,
                               float* __restrict__ in_om) {
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < m; e += gridDim.x * blockDim.x) {
    uint32_t s = src[e], d = dst[e];
    if (s == d) continue;  // a self-loop never improves D[s][v] (latency >= 1)
    float om = __fsub_rn(1.0f, loss[e]);
    uint32_t p = atomicAdd(&cursor[d], 1u);
    in_src[p] = s;
    in_lat[p] = lat[e];
    in_om[p] = om;
    if (!directed) {
      uint32_t q = atomicAdd(&cursor[s], 1u);
      in_src[q] = d;
      in_lat[q] = lat[e];
      in_om[q] = om;
    }
  }
}

// ---------------------------------------------------------------------------
// Packed-key batched relaxation, B sources per batch.
//
// Slab layout D[batch][node][B] (u64 keys).  With B = 32 a batch's slab is
// n x 256 B -- 2.56 MB at n = 10k, inside one XCD's 4 MB L2.  A wave owns
// G = 64 / B destination nodes (one per B-lane group; lane % B = source).
//
// XCD-aware 1-D grid: dispatch deals blocks round-robin over the 8 XCDs
// (MI355X_MICROARCH.md, "Workgroup dispatch"), so block L runs on XCD L % 8.
// Block L serves batch (L % 8) + 8 * ((L / 8) / nvb) and node chunk
// (L / 8) % nvb: every block of a batch lands on the same XCD, whose L2 then
// holds the batch's slab.  Placement changes speed only, never results.
//
// Frontier: dirty[batch][node] bytes mark nodes whose key changed in the
// previous pass (dprev) or earlier in this pass (dcur, read racily).  Arc
// (u -> v) is relaxed only if u is dirty.  Exactness: every change of u sets
// dcur[u]; in the next pass every out-neighbour re-reads u (across a kernel
// boundary, so the value is visible), and the iteration stops only after a
// pass with no change anywhere -- which is then the fixed point.
// ---------------------------------------------------------------------------
struct BatchMap {
  uint32_t nvb, n_batches;
  __device__ __forceinline__ bool decode(uint32_t L, uint32_t& batch, uint32_t& chunk) const {
    const uint32_t x = L & 7, k = L >> 3;
    batch = x + 8 * (k / nvb);
    chunk = k % nvb;
    return batch < n_batches;
  }
};

template <int B>
__global__ void k_init_front(uint64_t* __restrict__ D, uint32_t n, const uint32_t* __restrict__ used,
                             uint32_t first_row, uint32_t row_end, uint32_t n_batches) {
  const size_t total = (size_t)n_batches * n * B;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t s = (uint32_t)(i % B);
    const size_t bv = i / B;
    const uint32_t v = (uint32_t)(bv % n);
    const uint32_t b = (uint32_t)(bv / n);
    const uint32_t row = first_row + b * B + s;
    D[i] = (row < row_end && used[row] == v) ? 0ull : KEY_INF;  // PathProperties::default()
  }
}

template <int B, class FT>
__global__ void k_mark_sources(FT* __restrict__ dirty, uint32_t n, const uint32_t* __restrict__ used,
                               uint32_t first_row, uint32_t row_end, uint32_t n_batches) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_batches * B) return;
  const uint32_t b = t / B, row = first_row + t;
  if (row < row_end) dirty[(size_t)b * n + used[row]] = 1;
}

template <int B, int VPW, bool XCD, bool FLAGS>
__global__ void __launch_bounds__(RELAX_BLOCK)
    k_relax_front(const uint32_t* __restrict__ in_off, const uint32_t* __restrict__ in_src,
                  const uint64_t* __restrict__ in_lat, const float* __restrict__ in_om, uint64_t* D,
                  uint32_t n, BatchMap map, const uint32_t* __restrict__ active,
                  uint32_t* __restrict__ changed, const uint8_t* dprev, uint8_t* dcur,
                  unsigned long long* __restrict__ work) {
  constexpr int G = 64 / B;
  constexpr int NB = RELAX_WAVES * G * VPW;  // destination nodes per block
  // Staged in-arcs of the block's nodes: source (bit 31 = source is dirty),
  // clamped latency, 1 - loss.  Loaded coalesced, so the inner loop's only
  // global access is the independent distance-row read of each dirty arc.
  __shared__ uint32_t s_u[ARC_CHUNK];
  __shared__ uint64_t s_lat[ARC_CHUNK];
  __shared__ float s_om[ARC_CHUNK];
  __shared__ unsigned long long wblk[RELAX_WAVES];
  uint32_t b, chunk;
  if (XCD) {
    if (!map.decode(blockIdx.x, b, chunk) || !active[b]) return;
  } else {
    b = blockIdx.x / map.nvb;
    chunk = blockIdx.x % map.nvb;
    if (b >= map.n_batches || !active[b]) return;
  }
  uint64_t* Db = D + (size_t)b * n * B;
  const uint8_t* Pf = dprev + (size_t)b * n;
  uint8_t* Cf = dcur + (size_t)b * n;
  const int lane = threadIdx.x & 63;
  const int g = lane / B, s = lane % B;
  const uint32_t wave = threadIdx.x >> 6;
  const uint64_t gmask = (B == 64) ? ~0ull : (((1ull << (B & 63)) - 1) << (g * B));
  const uint32_t v0 = chunk * NB;
  const uint32_t vq = v0 + (wave * G + g) * VPW;  // this lane group's first node
  uint32_t lo[VPW], hi[VPW];
  uint64_t cur[VPW], best[VPW];
#pragma unroll
  for (int k = 0; k < VPW; k++) {
    const uint32_t v = vq + k;
    const bool valid = v < n;
    lo[k] = valid ? in_off[v] : 0;
    hi[k] = valid ? in_off[v + 1] : 0;
    cur[k] = valid ? Db[(size_t)v * B + s] : KEY_INF;
    best[k] = cur[k];
  }
  const uint32_t a_begin = in_off[v0], a_end = in_off[min(v0 + NB, n)];
  uint32_t n_relax = 0;
  for (uint32_t c0 = a_begin; c0 < a_end; c0 += ARC_CHUNK) {
    const uint32_t c1 = min(c0 + ARC_CHUNK, a_end);
    for (uint32_t a = c0 + threadIdx.x; a < c1; a += RELAX_BLOCK) {
      const uint32_t u = in_src[a];
      const bool f = !FLAGS || (Pf[u] | Cf[u]);
      s_u[a - c0] = u | (f ? 0x80000000u : 0u);
      s_lat[a - c0] = min(in_lat[a], LAT_SAT);
      s_om[a - c0] = in_om[a];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < VPW; k++) {
      uint32_t a = max(lo[k], c0);
      const uint32_t e = min(hi[k], c1);
      uint64_t bk = best[k];
      for (; a + 4 <= e; a += 4) {
        const uint32_t x0 = s_u[a - c0], x1 = s_u[a + 1 - c0], x2 = s_u[a + 2 - c0], x3 = s_u[a + 3 - c0];
        const size_t own = (size_t)(vq + k) * B + s;  // clean arcs re-read the node's own row (L1 hit)
        const uint64_t k0 = Db[(x0 >> 31) ? (size_t)(x0 & 0x7fffffffu) * B + s : own];
        const uint64_t k1 = Db[(x1 >> 31) ? (size_t)(x1 & 0x7fffffffu) * B + s : own];
        const uint64_t k2 = Db[(x2 >> 31) ? (size_t)(x2 & 0x7fffffffu) * B + s : own];
        const uint64_t k3 = Db[(x3 >> 31) ? (size_t)(x3 & 0x7fffffffu) * B + s : own];
        n_relax += (x0 >> 31) + (x1 >> 31) + (x2 >> 31) + (x3 >> 31);
        const uint64_t l0 = s_lat[a - c0], l1 = s_lat[a + 1 - c0], l2 = s_lat[a + 2 - c0], l3 = s_lat[a + 3 - c0];
        const float o0 = s_om[a - c0], o1 = s_om[a + 1 - c0], o2 = s_om[a + 2 - c0], o3 = s_om[a + 3 - c0];
        const uint64_t c0k = ((x0 >> 31) && k0 != KEY_INF) ? relax_key(k0, l0, o0) : KEY_INF;
        const uint64_t c1k = ((x1 >> 31) && k1 != KEY_INF) ? relax_key(k1, l1, o1) : KEY_INF;
        const uint64_t c2k = ((x2 >> 31) && k2 != KEY_INF) ? relax_key(k2, l2, o2) : KEY_INF;
        const uint64_t c3k = ((x3 >> 31) && k3 != KEY_INF) ? relax_key(k3, l3, o3) : KEY_INF;
        bk = min(bk, min(min(c0k, c1k), min(c2k, c3k)));
      }
      for (; a < e; a++) {
        const uint32_t x = s_u[a - c0];
        if (!(x >> 31)) continue;
        n_relax++;
        const uint64_t ku = Db[(size_t)(x & 0x7fffffffu) * B + s];
        if (ku != KEY_INF) bk = min(bk, relax_key(ku, s_lat[a - c0], s_om[a - c0]));
      }
      best[k] = bk;
    }
    __syncthreads();
  }
  bool any = false;
#pragma unroll
  for (int k = 0; k < VPW; k++) {
    const uint32_t v = vq + k;
    const bool ch = v < n && best[k] < cur[k];
    if (ch) Db[(size_t)v * B + s] = best[k];  // one untorn 64-bit (lat, loss) update
    const uint64_t m = __ballot(ch) & gmask;
    if (m && s == 0) Cf[v] = 1;
    any |= ch;
  }
  // every writer stores the same 1: a plain store, no same-address atomic storm
  if (__any(any) && lane == 0) __hip_atomic_store(&changed[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (work) {  // measurement only (timers on): block reduction, one add per block into a sharded counter
    unsigned long long wsum = n_relax;
    for (int d = 32; d > 0; d >>= 1) wsum += __shfl_xor(wsum, d, 64);
    if (lane == 0) wblk[wave] = wsum;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long t = 0;
      for (int w = 0; w < RELAX_WAVES; w++) t += wblk[w];
      if (t) atomicAdd(&work[blockIdx.x & (WORK_SHARDS - 1)], t);
    }
  }
}

// Wave-per-node relaxation (B = 64: lane = source).  The destination node is
// wave-uniform, so in-arcs and frontier flags are scalar loads; each dirty
// arc costs one coalesced 512-B row read.  Clean arcs read the node's own row
// instead (an L1 hit), keeping the four loads per step branch-free and in
// flight together.  Linear batch-major grid: all CUs work on the same one or
// two batches, whose slab rows stay hot in L2 / Infinity Cache.
template <int VPW, bool FLAGS, bool COUNT, bool XCD = false>
__global__ void __launch_bounds__(RELAX_BLOCK)
    k_relax_wave(const uint32_t* __restrict__ in_off, const uint32_t* __restrict__ in_src,
                 const uint64_t* __restrict__ in_lat, const float* __restrict__ in_om,
                 uint64_t* __restrict__ D, uint32_t n, const uint32_t* __restrict__ active,
                 uint32_t* __restrict__ changed, const uint32_t* dprev, uint32_t* dcur,
                 unsigned long long* __restrict__ work, uint32_t nvb = 0, uint32_t n_batches = 0) {
  constexpr int B = 64;
  uint32_t b, chunk;
  if (XCD) {  // 1-D grid: block L on XCD L % 8 serves batch (L % 8) + 8 * ((L / 8) / nvb)
    const uint32_t x = blockIdx.x & 7, q = blockIdx.x >> 3;
    b = x + 8 * (q / nvb);
    chunk = q % nvb;
    if (b >= n_batches) return;
  } else {
    b = blockIdx.y;
    chunk = blockIdx.x;
  }
  if (!active[b]) return;
  uint64_t* __restrict__ Db = D + (size_t)b * n * B;
  const uint32_t* Pf = dprev + (size_t)b * n;
  uint32_t* Cf = dcur + (size_t)b * n;
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  bool any = false;
  uint32_t n_relax = 0;  // wave-uniform count of dirty arcs (COUNT builds only)
  const uint32_t v0 = (chunk * RELAX_WAVES + wave) * VPW;
#pragma unroll 1
  for (int k = 0; k < VPW; k++) {
    const uint32_t v = v0 + k;
    if (v >= n) break;
    const uint32_t a0 = in_off[v], a1 = in_off[v + 1];
    const size_t own = (size_t)v * B + lane;
    const uint64_t cur = Db[own];
    uint64_t best = cur;
    uint32_t a = a0;
    // 4 independent 512-B row reads in flight per wave
    for (; a + 4 <= a1; a += 4) {
      const uint32_t u0 = in_src[a], u1 = in_src[a + 1], u2 = in_src[a + 2], u3 = in_src[a + 3];
      bool f0 = true, f1 = true, f2 = true, f3 = true;
      if (FLAGS) {  // clean sources re-read the node's own row (an L1 hit): branch-free loads
        f0 = (Pf[u0] | Cf[u0]) != 0;
        f1 = (Pf[u1] | Cf[u1]) != 0;
        f2 = (Pf[u2] | Cf[u2]) != 0;
        f3 = (Pf[u3] | Cf[u3]) != 0;
      }
      if (COUNT) n_relax += (uint32_t)f0 + (uint32_t)f1 + (uint32_t)f2 + (uint32_t)f3;
      const uint64_t k0 = Db[f0 ? (size_t)u0 * B + lane : own];
      const uint64_t k1 = Db[f1 ? (size_t)u1 * B + lane : own];
      const uint64_t k2 = Db[f2 ? (size_t)u2 * B + lane : own];
      const uint64_t k3 = Db[f3 ? (size_t)u3 * B + lane : own];
      const uint64_t l0 = min(in_lat[a], LAT_SAT), l1 = min(in_lat[a + 1], LAT_SAT);
      const uint64_t l2 = min(in_lat[a + 2], LAT_SAT), l3 = min(in_lat[a + 3], LAT_SAT);
      const float o0 = in_om[a], o1 = in_om[a + 1], o2 = in_om[a + 2], o3 = in_om[a + 3];
      const uint64_t c0 = (!f0 || k0 == KEY_INF) ? KEY_INF : relax_key(k0, l0, o0);
      const uint64_t c1 = (!f1 || k1 == KEY_INF) ? KEY_INF : relax_key(k1, l1, o1);
      const uint64_t c2 = (!f2 || k2 == KEY_INF) ? KEY_INF : relax_key(k2, l2, o2);
      const uint64_t c3 = (!f3 || k3 == KEY_INF) ? KEY_INF : relax_key(k3, l3, o3);
      best = min(best, min(min(c0, c1), min(c2, c3)));
    }
    for (; a < a1; a++) {
      const uint32_t u = in_src[a];
      const bool f = !FLAGS || (Pf[u] | Cf[u]) != 0;
      if (COUNT) n_relax += f;
      const uint64_t ku = Db[f ? (size_t)u * B + lane : own];
      const uint64_t l = min(in_lat[a], LAT_SAT);
      const float o = in_om[a];
      const uint64_t c = (!f || ku == KEY_INF) ? KEY_INF : relax_key(ku, l, o);
      best = min(best, c);
    }
    if (best < cur) {
      Db[own] = best;  // one untorn 64-bit (lat, loss) update
      any = true;
    }
    if (FLAGS && __any(best < cur) && lane == 0) Cf[v] = 1u;
  }
  if (__any(any) && lane == 0) atomicOr(&changed[b], 1u);
  if (COUNT && lane == 0 && n_relax) atomicAdd(&work[(blockIdx.x + blockIdx.y) & (WORK_SHARDS - 1)],
                                              (unsigned long long)n_relax * B);
}


// B = 32 sources per batch, two half-waves on adjacent destination nodes.
// XCD=true: block L runs batch (L % 8) + 8 * ((L / 8) / nvb) so every block of
// a batch shares an XCD (round-robin dispatch) and its 2.56 MB slab stays in
// that XCD's 4 MB L2.  Load scheduling as in the wave kernel: weights loaded
// unconditionally, row loads branch-free (clean arcs re-read the own row).
template <int VPW, bool XCD, bool FLAGS, bool COUNT>
__global__ void __launch_bounds__(RELAX_BLOCK)
    k_relax_half(const uint32_t* __restrict__ in_off, const uint32_t* __restrict__ in_src,
                 const uint64_t* __restrict__ in_lat, const float* __restrict__ in_om,
                 uint64_t* __restrict__ D, uint32_t n, uint32_t nvb, uint32_t n_batches,
                 const uint32_t* __restrict__ active, uint32_t* __restrict__ changed,
                 const uint32_t* dprev, uint32_t* dcur, unsigned long long* __restrict__ work) {
  constexpr int B = 32;
  uint32_t b, chunk;
  if (XCD) {
    const uint32_t x = blockIdx.x & 7, q = blockIdx.x >> 3;
    b = x + 8 * (q / nvb);
    chunk = q % nvb;
  } else {
    b = blockIdx.x / nvb;
    chunk = blockIdx.x % nvb;
  }
  if (b >= n_batches || !active[b]) return;
  uint64_t* __restrict__ Db = D + (size_t)b * n * B;
  const uint32_t* Pf = dprev + (size_t)b * n;
  uint32_t* Cf = dcur + (size_t)b * n;
  const int lane = threadIdx.x & 63;
  const int g = lane >> 5, s = lane & 31;
  const uint32_t wave = threadIdx.x >> 6;
  bool any = false;
  uint32_t n_relax = 0;
  const uint32_t v0 = (chunk * RELAX_WAVES + wave) * (2 * VPW);
#pragma unroll 1
  for (int k = 0; k < VPW; k++) {
    const uint32_t v = v0 + 2 * k + g;
    const bool valid = v < n;
    const uint32_t a0 = valid ? in_off[v] : 0, a1 = valid ? in_off[v + 1] : 0;
    const size_t own = valid ? (size_t)v * B + s : (size_t)s;
    const uint64_t cur = valid ? Db[own] : KEY_INF;
    uint64_t best = cur;
    uint32_t a = a0;
    for (; a + 4 <= a1; a += 4) {
      const uint32_t u0 = in_src[a], u1 = in_src[a + 1], u2 = in_src[a + 2], u3 = in_src[a + 3];
      bool f0 = true, f1 = true, f2 = true, f3 = true;
      if (FLAGS) {
        f0 = (Pf[u0] | Cf[u0]) != 0;
        f1 = (Pf[u1] | Cf[u1]) != 0;
        f2 = (Pf[u2] | Cf[u2]) != 0;
        f3 = (Pf[u3] | Cf[u3]) != 0;
      }
      if (COUNT) n_relax += (uint32_t)f0 + (uint32_t)f1 + (uint32_t)f2 + (uint32_t)f3;
      const uint64_t k0 = Db[f0 ? (size_t)u0 * B + s : own];
      const uint64_t k1 = Db[f1 ? (size_t)u1 * B + s : own];
      const uint64_t k2 = Db[f2 ? (size_t)u2 * B + s : own];
      const uint64_t k3 = Db[f3 ? (size_t)u3 * B + s : own];
      const uint64_t l0 = min(in_lat[a], LAT_SAT), l1 = min(in_lat[a + 1], LAT_SAT);
      const uint64_t l2 = min(in_lat[a + 2], LAT_SAT), l3 = min(in_lat[a + 3], LAT_SAT);
      const float o0 = in_om[a], o1 = in_om[a + 1], o2 = in_om[a + 2], o3 = in_om[a + 3];
      const uint64_t c0 = (!f0 || k0 == KEY_INF) ? KEY_INF : relax_key(k0, l0, o0);
      const uint64_t c1 = (!f1 || k1 == KEY_INF) ? KEY_INF : relax_key(k1, l1, o1);
      const uint64_t c2 = (!f2 || k2 == KEY_INF) ? KEY_INF : relax_key(k2, l2, o2);
      const uint64_t c3 = (!f3 || k3 == KEY_INF) ? KEY_INF : relax_key(k3, l3, o3);
      best = min(best, min(min(c0, c1), min(c2, c3)));
    }
    for (; a < a1; a++) {
      const uint32_t u = in_src[a];
      const bool f = !FLAGS || (Pf[u] | Cf[u]) != 0;
      if (COUNT) n_relax += f;
      const uint64_t ku = Db[f ? (size_t)u * B + s : own];
      const uint64_t l = min(in_lat[a], LAT_SAT);
      const float o = in_om[a];
      const uint64_t c = (!f || ku == KEY_INF) ? KEY_INF : relax_key(ku, l, o);
      best = min(best, c);
    }
    const bool ch = valid && best < cur;
    if (ch) {
      Db[own] = best;  // one untorn 64-bit (lat, loss) update
      any = true;
    }
    if (FLAGS) {
      const uint64_t m = __ballot(ch) >> (32 * g);
      if ((m & 0xffffffffull) && s == 0) Cf[v] = 1u;
    }
  }
  if (__any(any) && lane == 0) atomicOr(&changed[b], 1u);
  if (COUNT) {
    unsigned long long w = n_relax;
    for (int d = 32; d > 0; d >>= 1) w += __shfl_xor(w, d, 64);
    if (lane == 0 && w) atomicAdd(&work[blockIdx.x & (WORK_SHARDS - 1)], w);
  }
}

// Verbatim v1 relaxation kernel (A/B control, variant "v1k").
template <int VPW>
__global__ void __launch_bounds__(RELAX_BLOCK)
    k_relax_v1(const uint32_t* __restrict__ in_off, const uint32_t* __restrict__ in_src,
                   const uint64_t* __restrict__ in_lat, const float* __restrict__ in_om,
                   uint64_t* __restrict__ D, uint32_t n, const uint32_t* __restrict__ active,
                   uint32_t* __restrict__ changed) {
  const uint32_t b = blockIdx.y;
  if (!active[b]) return;
  uint64_t* __restrict__ Db = D + (size_t)b * n * BATCH;
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  bool any = false;
  const uint32_t v0 = (blockIdx.x * RELAX_WAVES + wave) * VPW;
#pragma unroll 1
  for (int k = 0; k < VPW; k++) {
    const uint32_t v = v0 + k;
    if (v >= n) break;
    const uint32_t a0 = in_off[v], a1 = in_off[v + 1];
    const uint64_t cur = Db[(size_t)v * BATCH + lane];
    uint64_t best = cur;
    uint32_t a = a0;
    // 4 independent 512-B row reads in flight per wave
    for (; a + 4 <= a1; a += 4) {
      uint32_t u0 = in_src[a], u1 = in_src[a + 1], u2 = in_src[a + 2], u3 = in_src[a + 3];
      uint64_t k0 = Db[(size_t)u0 * BATCH + lane];
      uint64_t k1 = Db[(size_t)u1 * BATCH + lane];
      uint64_t k2 = Db[(size_t)u2 * BATCH + lane];
      uint64_t k3 = Db[(size_t)u3 * BATCH + lane];
      uint64_t l0 = min(in_lat[a], LAT_SAT), l1 = min(in_lat[a + 1], LAT_SAT);
      uint64_t l2 = min(in_lat[a + 2], LAT_SAT), l3 = min(in_lat[a + 3], LAT_SAT);
      float o0 = in_om[a], o1 = in_om[a + 1], o2 = in_om[a + 2], o3 = in_om[a + 3];
      uint64_t c0 = k0 == KEY_INF ? KEY_INF : relax_key(k0, l0, o0);
      uint64_t c1 = k1 == KEY_INF ? KEY_INF : relax_key(k1, l1, o1);
      uint64_t c2 = k2 == KEY_INF ? KEY_INF : relax_key(k2, l2, o2);
      uint64_t c3 = k3 == KEY_INF ? KEY_INF : relax_key(k3, l3, o3);
      best = min(best, min(min(c0, c1), min(c2, c3)));
    }
    for (; a < a1; a++) {
      uint32_t u = in_src[a];
      uint64_t ku = Db[(size_t)u * BATCH + lane];
      uint64_t c = ku == KEY_INF ? KEY_INF : relax_key(ku, min(in_lat[a], LAT_SAT), in_om[a]);
      best = min(best, c);
    }
    if (best < cur) {
      Db[(size_t)v * BATCH + lane] = best;  // one untorn 64-bit (lat, loss) update
      any = true;
    }
  }
  if (__any(any) && lane == 0) atomicOr(&changed[b], 1u);
}

// Transposed write-out of [B rows x 64 cols] tiles.  Diagonal = the raw
// self-loop (graph/mod.rs:210-217).  Saturated keys flag their batch.
template <int B>
__global__ void __launch_bounds__(256)
    k_out_front(const uint64_t* __restrict__ D, uint32_t n, const uint32_t* __restrict__ used,
                uint32_t n_used, uint32_t first_row, uint32_t row_end, uint32_t out_row0,
                const uint32_t* __restrict__ self_edge, const uint64_t* __restrict__ e_lat,
                const float* __restrict__ e_loss, uint64_t* __restrict__ out_lat,
                float* __restrict__ out_loss, uint32_t* __restrict__ sat) {
  constexpr int G = 64 / B;
  __shared__ uint64_t tile[64][B + 1];
  const uint32_t b = blockIdx.y;
  const uint32_t j0 = blockIdx.x * 64;
  const uint64_t* __restrict__ Db = D + (size_t)b * n * B;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane / B, s = lane % B;
  for (int c = wave * G + g; c < 64; c += 4 * G) {
    const uint32_t j = j0 + c;
    tile[c][s] = j < n_used ? Db[(size_t)used[j] * B + s] : 0ull;
  }
  __syncthreads();
  bool sflag = false;
  const uint32_t j = j0 + lane;
  for (int r = wave; r < B; r += 4) {
    const uint32_t row = first_row + b * B + r;
    if (row >= row_end || j >= n_used) continue;
    const size_t o = (size_t)(row - out_row0) * n_used + j;
    if (row == j) {
      const uint32_t e = self_edge[used[j]];
      out_lat[o] = e_lat[e];
      out_loss[o] = e_loss[e];
    } else {
      const uint64_t kk = tile[lane][r];
      const uint64_t lat = key_lat(kk);
      sflag |= lat >= LAT_SAT;
      out_lat[o] = lat;
      out_loss[o] = __uint_as_float(key_loss_bits(kk));
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
  if (__any(ch) && lane == 0) atomicOr(changed, 1u);
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

__global__ void k_min_u64(const uint64_t* __restrict__ x, size_t count,
                          unsigned long long* __restrict__ out) {
  unsigned long long m = ~0ull;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
       i += (size_t)gridDim.x * blockDim.x)
    m = min(m, (unsigned long long)x[i]);
  for (int d = 32; d > 0; d >>= 1) m = min(m, (unsigned long long)__shfl_xor(m, d, 64));
  if ((threadIdx.x & 63) == 0) atomicMin(out, m);
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

static void build_net(sg_ctx* ctx, const sg_graph* g, sg_net* net) {
  const uint32_t n = g->n_nodes, m = g->n_edges;
  if (m && (!g->edge_src || !g->edge_dst || !g->edge_latency_ns || !g->edge_packet_loss))
    throw Error(SG_ERR_INVALID_ARG, "null edge array");
  for (uint32_t e = 0; e < m; e++) {
    if (g->edge_src[e] >= n || g->edge_dst[e] >= n)
      throw Error(SG_ERR_INVALID_ARG, "edge " + std::to_string(e) + " endpoint out of range");
    float l = g->edge_packet_loss[e];
    if (!(l >= 0.0f && l <= 1.0f))  // graph/mod.rs:101-103 (NaN rejected too)
      throw Error(SG_ERR_INVALID_ARG, "Edge 'packet_loss' is not in the range [0,1]");
    if (g->edge_latency_ns[e] == 0)  // graph/mod.rs:105-107
      throw Error(SG_ERR_INVALID_ARG, "Edge 'latency' must not be 0");
  }
  net->ctx = ctx;
  net->n_nodes = n;
  net->n_edges = m;
  net->directed = g->directed != 0;
  if (g->node_gml_id) net->gml_id.assign(g->node_gml_id, g->node_gml_id + n);
  hipStream_t st = ctx->stream;
  net->e_src = dmalloc<uint32_t>(m);
  net->e_dst = dmalloc<uint32_t>(m);
  net->e_lat = dmalloc<uint64_t>(m);
  net->e_loss = dmalloc<float>(m);
  net->in_off = dmalloc<uint32_t>((size_t)n + 1);
  net->self_cnt = dmalloc<uint32_t>(n);
  net->self_edge = dmalloc<uint32_t>(n);
  if (m) {
    SG_HIP(hipMemcpyAsync(net->e_src, g->edge_src, m * 4ull, hipMemcpyHostToDevice, st));
    SG_HIP(hipMemcpyAsync(net->e_dst, g->edge_dst, m * 4ull, hipMemcpyHostToDevice, st));
    SG_HIP(hipMemcpyAsync(net->e_lat, g->edge_latency_ns, m * 8ull, hipMemcpyHostToDevice, st));
    SG_HIP(hipMemcpyAsync(net->e_loss, g->edge_packet_loss, m * 4ull, hipMemcpyHostToDevice, st));
  }
  uint32_t* indeg = ctx->r_misc.get<uint32_t>((size_t)n + 1);
  SG_HIP(hipMemsetAsync(indeg, 0, ((size_t)n + 1) * 4, st));
  SG_HIP(hipMemsetAsync(net->self_cnt, 0, (size_t)n * 4, st));
  SG_HIP(hipMemsetAsync(net->self_edge, 0, (size_t)n * 4, st));
  if (m) {
    hipLaunchKernelGGL(k_count_arcs, dim3(grid_for(m, 256, 8192)), dim3(256), 0, st, net->e_src,
                       net->e_dst, m, (int)net->directed, indeg, net->self_cnt, net->self_edge);
    SG_CHECK_LAUNCH();
  }
  exclusive_scan_u32(ctx, indeg, net->in_off, n);
  uint32_t n_arcs = 0;
  copy_to_host(ctx, &n_arcs, net->in_off + n, 4);
  net->n_arcs = n_arcs;
  net->in_src = dmalloc<uint32_t>(n_arcs);
  net->in_lat = dmalloc<uint64_t>(n_arcs);
  net->in_om = dmalloc<float>(n_arcs);
  if (n_arcs) {
    uint32_t* cursor = ctx->r_map.get<uint32_t>((size_t)n + 1);
    SG_HIP(hipMemcpyAsync(cursor, net->in_off, ((size_t)n + 1) * 4, hipMemcpyDeviceToDevice, st));
    hipLaunchKernelGGL(k_scatter_arcs, dim3(grid_for(m, 256, 8192)), dim3(256), 0, st, net->e_src,
                       net->e_dst, net->e_lat, net->e_loss, m, (int)net->directed, cursor,
                       net->in_src, net->in_lat, net->in_om);
    SG_CHECK_LAUNCH();
  }
  SG_HIP(hipStreamSynchronize(st));
}

static void check_self_loops(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used,
                             const uint32_t* h_used) {
  unsigned long long* first = ctx->r_err.get<unsigned long long>(4);
  SG_HIP(hipMemsetAsync(first, 0xff, 8, ctx->stream));
  hipLaunchKernelGGL(k_self_check, dim3(grid_for(n_used, 256, 4096)), dim3(256), 0, ctx->stream,
                     d_used, n_used, net->self_cnt, first);
  SG_CHECK_LAUNCH();
  unsigned long long h = 0;
  copy_to_host(ctx, &h, first, 8);
  if (h != ~0ull) {
    uint32_t j = (uint32_t)(h >> 1);
    std::string id = node_name(net, h_used[j]);
    if (h & 1)
      throw Error(SG_ERR_MULTI_EDGE, "More than one edge connecting node " + id + " to " + id, j, j);
    throw Error(SG_ERR_NO_EDGE, "No edge connecting node " + id + " to " + id, j, j);
  }
}

// Wide recomputation of the listed rows (absolute row indices).
static void run_wide(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used,
                     const std::vector<uint32_t>& rows, uint32_t out_row0, uint64_t* out_lat,
                     float* out_loss) {
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

template <int B, int VPW, bool XCD, bool FLAGS, bool WAVE, bool HALF = false>
static void shortest_paths_t(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used,
                             uint32_t row_begin, uint32_t row_end, uint64_t* out_lat,
                             float* out_loss) {
  // B = sources per batch (B = 32: slab n x 256 B, L2-resident per XCD at 10k nodes);
  // VPW = destination nodes per lane group, walked sequentially;
  // WAVE = wave-per-node kernel (B = 64, scalar arc loads, u32 frontier flags)
  static_assert(!WAVE || B == 64, "wave-per-node kernel needs B = 64");
  static_assert(!HALF || B == 32, "half-wave kernel needs B = 32");
  using FT = typename std::conditional<WAVE || HALF, uint32_t, uint8_t>::type;
  constexpr int G = 64 / B;
  hipStream_t st = ctx->stream;
  const uint32_t n = net->n_nodes;
  const uint32_t n_rows = row_end - row_begin;
  const uint32_t n_batches = (n_rows + B - 1) / B;
  // Group size: batches whose slabs are live together (bounded device memory).
  const size_t slab_bytes = (size_t)n * B * 8;
  const size_t budget = (size_t)env_int("SG_APSP_GROUP_MB", 4096) << 20;
  const uint32_t group = (uint32_t)std::max<size_t>(1, std::min<size_t>(n_batches, budget / slab_bytes));
  const uint32_t nvb = (n + RELAX_WAVES * G * VPW - 1) / (RELAX_WAVES * G * VPW);
  uint64_t* D = ctx->r_dist.get<uint64_t>((size_t)group * n * B);
  // per-batch flags: a 3-slot ring of "changed in pass p" arrays, then the saturation flags
  uint32_t* flags = ctx->r_flags.get<uint32_t>((size_t)group * 4 + 8);
  uint32_t* ring[3] = {flags, flags + group, flags + 2 * (size_t)group};
  uint32_t* sat = flags + 3 * (size_t)group;
  FT* dirty = ctx->r_dirty.get<FT>(2 * (size_t)group * n);
  FT* dirtyA[2] = {dirty, dirty + (size_t)group * n};
  unsigned long long* work = ctx->timing ? ctx->r_work.get<unsigned long long>(WORK_SHARDS) : nullptr;
  if (work) SG_HIP(hipMemsetAsync(work, 0, WORK_SHARDS * 8, st));
  // Passes are issued in chunks; the host reads the convergence flags once per
  // chunk.  A pass issued after its batch converged exits at once (active == 0).
  const uint32_t chunk = (uint32_t)std::max(1, env_int("SG_APSP_PASS_CHUNK", 4));
  std::vector<uint32_t> h_changed(group), h_sat(group);
  std::vector<uint32_t> wide_rows;
  for (uint32_t g0 = 0; g0 < n_batches; g0 += group) {
    const uint32_t gb = std::min(group, n_batches - g0);
    const uint32_t first_row = row_begin + g0 * B;
    hipLaunchKernelGGL(k_init_front<B>, dim3(grid_for((size_t)gb * n * B, 256, 65536)), dim3(256), 0, st, D, n,
                       d_used, first_row, row_end, gb);
    SG_HIP(hipMemsetAsync(dirty, 0, 2 * (size_t)gb * n * sizeof(FT), st));
    dirtyA[1] = dirty + (size_t)gb * n;
    hipLaunchKernelGGL((k_mark_sources<B, FT>), dim3(grid_for((size_t)gb * B, 256)), dim3(256), 0, st, dirtyA[1], n,
                       d_used, first_row, row_end, gb);
    SG_CHECK_LAUNCH();
    SG_HIP(hipMemsetAsync(ring[2], 1, gb * 4ull, st));  // "changed in pass -1": every batch active
    const BatchMap map{nvb, gb};
    const uint32_t grid = XCD ? 8 * nvb * ((gb + 7) / 8) : nvb * gb;
    for (uint32_t pass = 0;;) {
      uint32_t last = pass;
      for (uint32_t c = 0; c < chunk; c++, pass++) {
        if (pass > n + 2 + chunk) throw Error(SG_ERR_DEVICE, "relaxation did not converge");
        const uint32_t* active = ring[(pass + 2) % 3];
        uint32_t* changed = ring[pass % 3];
        FT* dcur = dirtyA[pass & 1];
        const FT* dprev = dirtyA[(pass & 1) ^ 1];
        SG_HIP(hipMemsetAsync(changed, 0, gb * 4ull, st));
        if (pass) SG_HIP(hipMemsetAsync(dcur, 0, (size_t)gb * n * sizeof(FT), st));
        {
          TimedLaunch tl(ctx, "relax_packed", 0.0);
          if (getenv("SG_APSP_V1K")) {
            const uint32_t nvb1 = (n + RELAX_WAVES * 4 - 1) / (RELAX_WAVES * 4);
            hipLaunchKernelGGL(k_relax_v1<4>, dim3(nvb1, gb), dim3(RELAX_BLOCK), 0, st, net->in_off, net->in_src,
                               net->in_lat, net->in_om, D, n, active, changed);
          } else if constexpr (HALF) {
            const uint32_t nvh = (n + RELAX_WAVES * 2 * VPW - 1) / (RELAX_WAVES * 2 * VPW);
            const uint32_t gridh = XCD ? 8 * nvh * ((gb + 7) / 8) : nvh * gb;
            if (work)
              hipLaunchKernelGGL((k_relax_half<VPW, XCD, FLAGS, true>), dim3(gridh), dim3(RELAX_BLOCK), 0, st,
                                 net->in_off, net->in_src, net->in_lat, net->in_om, D, n, nvh, gb, active, changed,
                                 (const uint32_t*)dprev, (uint32_t*)dcur, work);
            else
              hipLaunchKernelGGL((k_relax_half<VPW, XCD, FLAGS, false>), dim3(gridh), dim3(RELAX_BLOCK), 0, st,
                                 net->in_off, net->in_src, net->in_lat, net->in_om, D, n, nvh, gb, active, changed,
                                 (const uint32_t*)dprev, (uint32_t*)dcur, work);
          } else if constexpr (WAVE) {
            const uint32_t nvw = (n + RELAX_WAVES * VPW - 1) / (RELAX_WAVES * VPW);
            const dim3 gw = XCD ? dim3(8 * nvw * ((gb + 7) / 8)) : dim3(nvw, gb);
            if (work)
              hipLaunchKernelGGL((k_relax_wave<VPW, FLAGS, true, XCD>), gw, dim3(RELAX_BLOCK), 0, st,
                                 net->in_off, net->in_src, net->in_lat, net->in_om, D, n, active, changed,
                                 (const uint32_t*)dprev, (uint32_t*)dcur, work, nvw, gb);
            else
              hipLaunchKernelGGL((k_relax_wave<VPW, FLAGS, false, XCD>), gw, dim3(RELAX_BLOCK), 0, st,
                                 net->in_off, net->in_src, net->in_lat, net->in_om, D, n, active, changed,
                                 (const uint32_t*)dprev, (uint32_t*)dcur, work, nvw, gb);
          } else {
            hipLaunchKernelGGL((k_relax_front<B, VPW, XCD, FLAGS>), dim3(grid), dim3(RELAX_BLOCK), 0, st,
                               net->in_off, net->in_src, net->in_lat, net->in_om, D, n, map, active, changed,
                               (const uint8_t*)dprev, (uint8_t*)dcur, work);
          }
        }
        SG_CHECK_LAUNCH();
        last = pass;
      }
      copy_to_host(ctx, h_changed.data(), ring[last % 3], gb * 4ull);
      uint32_t n_active = 0;
      for (uint32_t b = 0; b < gb; b++) n_active += h_changed[b] != 0;
      if (!n_active) break;
    }
    SG_HIP(hipMemsetAsync(sat, 0, gb * 4ull, st));
    {
      TimedLaunch tl(ctx, "out_packed", 12.0 * std::min<uint32_t>(gb * B, row_end - first_row) * n_used);
      hipLaunchKernelGGL(k_out_front<B>, dim3((n_used + 63) / 64, gb), dim3(256), 0, st, D, n, d_used, n_used,
                         first_row, row_end, row_begin, net->self_edge, net->e_lat, net->e_loss, out_lat,
                         out_loss, sat);
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
  if (work) {  // relaxations actually performed (dirty arcs x lanes), for the roofline
    unsigned long long w[WORK_SHARDS];
    copy_to_host(ctx, w, work, sizeof(w));
    double total = 0;
    for (int k = 0; k < WORK_SHARDS; k++) total += (double)w[k];
    timer_add_work(ctx, "relax_packed", total);
  }
  if (!wide_rows.empty()) run_wide(ctx, net, d_used, n_used, wide_rows, row_begin, out_lat, out_loss);
}

// Kernel variant (A/B measurement): SG_APSP_VARIANT = "<B>[x][f]" (x = XCD-aware
// grid, f = frontier flags); default below.
static void shortest_paths(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used,
                           uint32_t row_begin, uint32_t row_end, uint64_t* out_lat, float* out_loss) {
  const char* v = getenv("SG_APSP_VARIANT");
  std::string var = v && *v ? v : "w64xv32";
#define SG_VAR(name, B, VPW, X, F, W)                                                                \
  if (var == name) {                                                                                 \
    shortest_paths_t<B, VPW, X, F, W>(ctx, net, d_used, n_used, row_begin, row_end, out_lat, out_loss); \
    return;                                                                                          \
  }
#define SG_VARH(name, VPW, X, F)                                                                     \
  if (var == name) {                                                                                 \
    shortest_paths_t<32, VPW, X, F, false, true>(ctx, net, d_used, n_used, row_begin, row_end, out_lat, \
                                                 out_loss);                                          \
    return;                                                                                          \
  }
  SG_VARH("h32x", 4, true, false)
  SG_VARH("h32xf", 4, true, true)
  SG_VARH("h32", 4, false, false)
  SG_VARH("h32xv2", 2, true, false)
  SG_VAR("w64x", 64, 4, true, false, true)
  SG_VAR("w64xf", 64, 4, true, true, true)
  SG_VAR("w64v8", 64, 8, false, false, true)
  SG_VAR("w64v16", 64, 16, false, false, true)
  SG_VAR("w64v32", 64, 32, false, false, true)
  SG_VAR("w64xv8", 64, 8, true, false, true)
  SG_VAR("w64xv16", 64, 16, true, false, true)
  SG_VAR("w64fv16", 64, 16, false, true, true)
  SG_VAR("w64v64", 64, 64, false, false, true)
  SG_VAR("w64v128", 64, 128, false, false, true)
  SG_VAR("w64xv32", 64, 32, true, false, true)
  SG_VAR("w64xv64", 64, 64, true, false, true)
  SG_VAR("w64f", 64, 4, false, true, true)
  SG_VAR("w64", 64, 4, false, false, true)
  SG_VAR("32xf", 32, 4, true, true, false)
  SG_VAR("32x", 32, 4, true, false, false)
  SG_VAR("32f", 32, 4, false, true, false)
  SG_VAR("32", 32, 4, false, false, false)
  SG_VAR("64xf", 64, 4, true, true, false)
  SG_VAR("64x", 64, 4, true, false, false)
  SG_VAR("64f", 64, 4, false, true, false)
  SG_VAR("64", 64, 4, false, false, false)
#undef SG_VAR
#undef SG_VARH
  throw Error(SG_ERR_INVALID_ARG, "unknown SG_APSP_VARIANT " + var);
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
  if (net->ctx) (void)hipSetDevice(net->ctx->device);
  delete net;
}

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
    {
      std::vector<uint8_t> seen(net->n_nodes, 0);
      for (uint32_t j = 0; j < n_used; j++) {
        if (nodes[j] >= net->n_nodes) throw Error(SG_ERR_INVALID_ARG, "node index out of range");
        if (seen[nodes[j]]++) throw Error(SG_ERR_INVALID_ARG, "duplicate node in node list");
      }
    }
    if (n_used == 0) return;
    hipStream_t st = ctx->stream;
    uint32_t* d_used = ctx->r_used.get<uint32_t>(n_used);
    SG_HIP(hipMemcpyAsync(d_used, nodes, (size_t)n_used * 4, hipMemcpyHostToDevice, st));
    const bool shortest = flags & SG_ROUTE_SHORTEST_PATH;
    // The reference checks every used node's self-loop (graph/mod.rs:211-217),
    // whichever rows this call computes.
    if (shortest) check_self_loops(ctx, net, d_used, n_used, nodes);
    if (row_end == row_begin) return;
    const size_t count = (size_t)(row_end - row_begin) * n_used;
    const bool dev_out = flags & SG_ROUTE_OUT_DEVICE;
    uint64_t* o_lat = dev_out ? out_latency_ns : ctx->r_out_lat.get<uint64_t>(count);
    float* o_loss = dev_out ? out_packet_loss : ctx->r_out_loss.get<float>(count);
    if (shortest)
      shortest_paths(ctx, net, d_used, n_used, row_begin, row_end, o_lat, o_loss);
    else
      direct_paths(ctx, net, d_used, nodes, n_used, row_begin, row_end, o_lat, o_loss);
    if (!dev_out) {
      SG_HIP(hipMemcpyAsync(out_latency_ns, o_lat, count * 8, hipMemcpyDeviceToHost, st));
      SG_HIP(hipMemcpyAsync(out_packet_loss, o_loss, count * 4, hipMemcpyDeviceToHost, st));
    }
    SG_HIP(hipStreamSynchronize(st));
  });
}

int32_t sg_routing_min_latency(sg_ctx* ctx, const uint64_t* d_latency_ns, size_t count,
                               uint64_t* out_min) {
  return sg::guarded(ctx, [&] {
    using namespace sg;
    if (!out_min || (count && !d_latency_ns)) throw Error(SG_ERR_INVALID_ARG, "null argument");
    unsigned long long* m = ctx->r_err.get<unsigned long long>(4);
    SG_HIP(hipMemsetAsync(m, 0xff, 8, ctx->stream));
    if (count)
      hipLaunchKernelGGL(k_min_u64, dim3(grid_for(count, 256, 4096)), dim3(256), 0, ctx->stream,
                         d_latency_ns, count, m);
    SG_CHECK_LAUNCH();
    unsigned long long h = 0;
    copy_to_host(ctx, &h, m, 8);
    *out_min = h;
  });
}

}  // extern "C"
