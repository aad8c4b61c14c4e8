// sg_route_info.hip -- the host half of the routing boundary: a dense RoutingInfo.
//
// The reference materialises the routing table twice as
// HashMap<(NodeIndex, NodeIndex), PathProperties> (compute_shortest_paths,
// graph/mod.rs:190-208) and HashMap<(u32, u32), PathProperties> (the id remap of
// generate_routing_info, sim_config.rs:423-445), n_used^2 entries each, and then
// answers every RoutingInfo::path (graph/mod.rs:448-450) with a SipHash lookup --
// two per sent packet (WorkerShared::latency / reliability, worker.rs:517-531)
// plus the legacy C TCP's worker_getLatency (worker.rs:651-661, tcp.c:448).
//
// Here the table is one row-major array of 8-byte cells (latency u32 << 32 |
// bits(loss)) in pinned host memory (the D2H target of sg_routing_info_fill,
// sg_routing.hip), keyed by a GML-id -> row map and an address -> row map
// (IpAssignment::get_node, graph/mod.rs:397-399), so a lookup is two array reads
// and no hashing.  A path of 2^32 - 1 ns (4.29 s) or more keeps its u64 latency
// in a sorted side table (its cell says SG_CELL_WIDE); the reference's u64
// latency is kept exactly either way.
// Lookups are read-only; packet counters are atomic (the reference takes a
// global RwLock write per packet, graph/mod.rs:453-460).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "sg_internal.h"

sg_routing_info::~sg_routing_info() {
  if (pinned) {
    if (cell) (void)hipHostFree(cell);
  } else {
    free(cell);
  }
  free(counters.load());
}

namespace sg {

// key -> value map over u32 keys: a dense window when the keys are compact
// (Shadow numbers GML nodes 0.. and assigns addresses 11.0.0.1.. in order),
// else sorted pairs and a binary search.
static void build_map(const uint32_t* keys, const uint32_t* vals, uint32_t n, uint32_t& base, uint32_t& span,
                      std::vector<uint32_t>& dense, std::vector<std::pair<uint32_t, uint32_t>>& sorted,
                      const char* what) {
  dense.clear();
  sorted.clear();
  base = span = 0;
  if (!n) return;
  uint32_t lo = keys[0], hi = keys[0];
  for (uint32_t i = 1; i < n; i++) {
    lo = std::min(lo, keys[i]);
    hi = std::max(hi, keys[i]);
  }
  const uint64_t width = (uint64_t)hi - lo + 1;
  if (width <= 4ull * n + 1024) {
    base = lo;
    span = (uint32_t)width;
    dense.assign(span, ~0u);
    for (uint32_t i = 0; i < n; i++) {
      uint32_t& slot = dense[keys[i] - lo];
      if (slot != ~0u) throw Error(SG_ERR_INVALID_ARG, std::string("duplicate ") + what);
      slot = vals[i];
    }
  } else {
    sorted.resize(n);
    for (uint32_t i = 0; i < n; i++) sorted[i] = {keys[i], vals[i]};
    std::sort(sorted.begin(), sorted.end());
    for (uint32_t i = 1; i < n; i++)
      if (sorted[i].first == sorted[i - 1].first) throw Error(SG_ERR_INVALID_ARG, std::string("duplicate ") + what);
  }
}

static inline uint32_t map_get(uint32_t key, uint32_t base, uint32_t span, const std::vector<uint32_t>& dense,
                               const std::vector<std::pair<uint32_t, uint32_t>>& sorted) {
  if (span) {
    const uint32_t k = key - base;
    return k < span ? dense[k] : ~0u;
  }
  auto it = std::lower_bound(sorted.begin(), sorted.end(), std::make_pair(key, 0u));
  return it != sorted.end() && it->first == key ? it->second : ~0u;
}

static inline uint32_t row_of(const sg_routing_info* ri, uint32_t id) {
  return map_get(id, ri->id_base, ri->id_span, ri->id_dense, ri->id_sorted);
}

// an assigned address whose node has no routing row (is_routable still holds)
constexpr uint32_t ROW_UNROUTED = 0xFFFFFFFEu;

static inline uint32_t row_of_ip_be(const sg_routing_info* ri, uint32_t ip_be) {
  return map_get(__builtin_bswap32(ip_be), ri->ip_base, ri->ip_span, ri->ip_dense, ri->ip_sorted);
}

// cell c -> (latency, loss)
static inline void cell_get(const sg_routing_info* ri, size_t c, uint64_t* lat, float* loss) {
  const uint64_t x = ri->cell[c];
  if (loss) {
    const uint32_t b = (uint32_t)x;
    memcpy(loss, &b, 4);
  }
  if (!lat) return;
  if ((x >> 32) != SG_CELL_WIDE) {
    *lat = x >> 32;
    return;
  }
  auto it = std::lower_bound(ri->wide.begin(), ri->wide.end(), (uint64_t)c,
                             [](const sg_routing_info::Wide& w, uint64_t k) { return w.cell < k; });
  *lat = it != ri->wide.end() && it->cell == c ? it->lat : UINT64_MAX;
}

static void* host_alloc(size_t bytes, bool& pinned) {
  // pinned (the DMA target of sg_routing_info_fill) when a HIP device is present
  int count = 0;
  if (hipGetDeviceCount(&count) == hipSuccess && count > 0) {
    void* p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(bytes, 16), hipHostMallocDefault) == hipSuccess) {
      pinned = true;
      return p;
    }
  }
  pinned = false;
  void* p = aligned_alloc(64, (std::max<size_t>(bytes, 16) + 63) & ~(size_t)63);
  if (!p) throw std::bad_alloc();
  return p;
}

}  // namespace sg

extern "C" {

int32_t sg_routing_info_create(uint32_t n_used, const uint32_t* node_ids, sg_routing_info** out) {
  if (!out || (n_used && !node_ids)) return SG_ERR_INVALID_ARG;
  *out = nullptr;
  sg_routing_info* ri = nullptr;
  try {
    ri = new sg_routing_info();
    ri->n = n_used;
    ri->node_ids.assign(node_ids, node_ids + n_used);
    std::vector<uint32_t> rows(n_used);
    for (uint32_t i = 0; i < n_used; i++) rows[i] = i;
    sg::build_map(node_ids, rows.data(), n_used, ri->id_base, ri->id_span, ri->id_dense, ri->id_sorted,
                  "node id");
    const size_t cells = (size_t)n_used * n_used;
    ri->cell = (uint64_t*)sg::host_alloc(cells * 8, ri->pinned);
    ri->row_set.assign(n_used, 0);
    ri->row_min.assign(n_used, UINT64_MAX);
  } catch (const sg::Error& e) {
    delete ri;
    return e.code;
  } catch (...) {
    delete ri;
    return SG_ERR_OOM;
  }
  *out = ri;
  return SG_OK;
}

void sg_routing_info_destroy(sg_routing_info* ri) { delete ri; }

int32_t sg_routing_info_set_rows(sg_routing_info* ri, uint32_t row_begin, uint32_t row_end,
                                 const uint64_t* latency_ns, const float* packet_loss) {
  if (!ri || row_begin > row_end || row_end > ri->n) return SG_ERR_INVALID_ARG;
  if (row_end > row_begin && (!latency_ns || !packet_loss)) return SG_ERR_INVALID_ARG;
  try {
    const size_t off = (size_t)row_begin * ri->n, cells = (size_t)(row_end - row_begin) * ri->n;
    // rows written again drop their old wide entries
    auto lo = std::lower_bound(ri->wide.begin(), ri->wide.end(), (uint64_t)off,
                               [](const sg_routing_info::Wide& w, uint64_t k) { return w.cell < k; });
    auto hi = std::lower_bound(lo, ri->wide.end(), (uint64_t)(off + cells),
                               [](const sg_routing_info::Wide& w, uint64_t k) { return w.cell < k; });
    std::vector<sg_routing_info::Wide> add;
    const uint32_t n = ri->n;
    for (uint32_t r = row_begin; r < row_end; r++) {
      uint64_t rm = UINT64_MAX;
      for (uint32_t c = 0; c < n; c++) {
        const size_t i = (size_t)(r - row_begin) * n + c;
        uint32_t b;
        memcpy(&b, &packet_loss[i], 4);
        const uint64_t l = latency_ns[i];
        const uint32_t hi32 = l < SG_CELL_WIDE ? (uint32_t)l : SG_CELL_WIDE;
        ri->cell[off + i] = ((uint64_t)hi32 << 32) | b;
        if (hi32 == SG_CELL_WIDE) add.push_back({off + i, l});
        rm = std::min(rm, l);
      }
      ri->rows_set += ri->row_set[r] ? 0u : 1u;
      ri->row_set[r] = 1;
      ri->row_min[r] = rm;
    }
    const size_t at = lo - ri->wide.begin();
    ri->wide.erase(lo, hi);
    ri->wide.insert(ri->wide.begin() + at, add.begin(), add.end());
    // get_smallest_latency_ns (graph/mod.rs:478-480) is over every entry: once the whole
    // table is present, the smallest of the per-row minima (rows may have been rewritten;
    // a row a fill wrote gets its minimum once, from its cells and the side table)
    if (ri->rows_set == n) {
      uint64_t m = UINT64_MAX;
      for (uint32_t r = 0; r < n; r++) {
        if (ri->row_set[r] == 2) {
          const size_t o = (size_t)r * n;
          uint64_t rm = UINT64_MAX;
          for (uint32_t c = 0; c < n; c++) rm = std::min(rm, ri->cell[o + c] >> 32);
          if (rm == SG_CELL_WIDE) {  // every cell of the row is wide: its smallest u64 latency
            rm = UINT64_MAX;
            auto w = std::lower_bound(ri->wide.begin(), ri->wide.end(), (uint64_t)o,
                                      [](const sg_routing_info::Wide& x, uint64_t k) { return x.cell < k; });
            for (; w != ri->wide.end() && w->cell < o + n; ++w) rm = std::min(rm, w->lat);
          }
          ri->row_min[r] = rm;
          ri->row_set[r] = 1;
        }
        m = std::min(m, ri->row_min[r]);
      }
      ri->min_lat = m;
      ri->filled = true;
    }
  } catch (...) {
    return SG_ERR_OOM;
  }
  return SG_OK;
}

int32_t sg_routing_info_view(const sg_routing_info* ri, sg_routing_view* out) {
  if (!ri || !out) return SG_ERR_INVALID_ARG;
  out->n = ri->n;
  out->node_ids = ri->node_ids.data();
  out->cells = ri->cell;
  out->n_wide = ri->wide.size();
  out->pinned = ri->pinned ? 1 : 0;
  return SG_OK;
}

int32_t sg_routing_info_rows(const sg_routing_info* ri, uint32_t row_begin, uint32_t row_end, uint64_t* latency_ns,
                             float* packet_loss) {
  if (!ri || row_begin > row_end || row_end > ri->n) return SG_ERR_INVALID_ARG;
  if (row_end > row_begin && (!latency_ns || !packet_loss)) return SG_ERR_INVALID_ARG;
  const size_t off = (size_t)row_begin * ri->n, cells = (size_t)(row_end - row_begin) * ri->n;
  for (size_t i = 0; i < cells; i++) {
    const uint64_t x = ri->cell[off + i];
    latency_ns[i] = x >> 32;
    const uint32_t b = (uint32_t)x;
    memcpy(&packet_loss[i], &b, 4);
  }
  auto it = std::lower_bound(ri->wide.begin(), ri->wide.end(), (uint64_t)off,
                             [](const sg_routing_info::Wide& w, uint64_t k) { return w.cell < k; });
  for (; it != ri->wide.end() && it->cell < off + cells; ++it) latency_ns[it->cell - off] = it->lat;
  return SG_OK;
}

int32_t sg_routing_info_index(const sg_routing_info* ri, uint32_t node_id, uint32_t* row) {
  if (!ri || !row) return SG_ERR_INVALID_ARG;
  const uint32_t r = sg::row_of(ri, node_id);
  if (r == ~0u) return SG_ERR_INVALID_ARG;
  *row = r;
  return SG_OK;
}

int32_t sg_routing_info_path(const sg_routing_info* ri, uint32_t start, uint32_t end, uint64_t* latency_ns,
                             float* packet_loss) {
  if (!ri) return 0;
  const uint32_t i = sg::row_of(ri, start), j = sg::row_of(ri, end);
  if (i == ~0u || j == ~0u) return 0;  // None
  sg::cell_get(ri, (size_t)i * ri->n + j, latency_ns, packet_loss);
  return 1;
}

int32_t sg_routing_info_smallest_latency(const sg_routing_info* ri, uint64_t* out) {
  if (!ri || !out || !ri->n || !ri->filled) return 0;  // None: no paths
  *out = ri->min_lat;
  return 1;
}

int32_t sg_routing_info_increment_packet_count(sg_routing_info* ri, uint32_t start, uint32_t end) {
  if (!ri) return SG_ERR_INVALID_ARG;
  const uint32_t i = sg::row_of(ri, start), j = sg::row_of(ri, end);
  if (i == ~0u || j == ~0u) return SG_ERR_INVALID_ARG;
  uint64_t* cnt = ri->counters.load(std::memory_order_acquire);
  if (!cnt) {
    uint64_t* fresh = (uint64_t*)calloc(std::max<size_t>((size_t)ri->n * ri->n, 1), 8);
    if (!fresh) return SG_ERR_OOM;
    uint64_t* expect = nullptr;
    if (ri->counters.compare_exchange_strong(expect, fresh, std::memory_order_acq_rel))
      cnt = fresh;
    else {
      free(fresh);
      cnt = expect;
    }
  }
  uint64_t* c = &cnt[(size_t)i * ri->n + j];
  uint64_t v = __atomic_load_n(c, __ATOMIC_RELAXED);
  while (v != UINT64_MAX && !__atomic_compare_exchange_n(c, &v, v + 1, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }  // saturating_add(1)
  return SG_OK;
}

uint64_t sg_routing_info_packet_count(const sg_routing_info* ri, uint32_t start, uint32_t end) {
  if (!ri) return 0;
  const uint32_t i = sg::row_of(ri, start), j = sg::row_of(ri, end);
  const uint64_t* cnt = ri->counters.load(std::memory_order_acquire);
  if (i == ~0u || j == ~0u || !cnt) return 0;
  return __atomic_load_n(&cnt[(size_t)i * ri->n + j], __ATOMIC_RELAXED);
}

int32_t sg_routing_info_set_addresses(sg_routing_info* ri, uint32_t n_addrs, const uint32_t* ipv4,
                                      const uint32_t* node_id) {
  if (!ri || (n_addrs && (!ipv4 || !node_id))) return SG_ERR_INVALID_ARG;
  try {
    std::vector<uint32_t> rows(n_addrs);
    for (uint32_t i = 0; i < n_addrs; i++) {
      const uint32_t r = sg::row_of(ri, node_id[i]);
      rows[i] = r == ~0u ? sg::ROW_UNROUTED : r;
    }
    sg::build_map(ipv4, rows.data(), n_addrs, ri->ip_base, ri->ip_span, ri->ip_dense, ri->ip_sorted, "address");
  } catch (const sg::Error& e) {
    return e.code == SG_ERR_INVALID_ARG ? SG_ERR_DUPLICATE_IP : e.code;
  } catch (...) {
    return SG_ERR_OOM;
  }
  return SG_OK;
}

int32_t sg_worker_get_latency(const sg_routing_info* ri, uint32_t src_be, uint32_t dst_be, uint64_t* latency_ns) {
  if (!ri || !latency_ns) return SG_ERR_INVALID_ARG;
  const uint32_t i = sg::row_of_ip_be(ri, src_be), j = sg::row_of_ip_be(ri, dst_be);
  if (i >= ri->n || j >= ri->n) return SG_ERR_INVALID_ARG;  // None (worker_getLatency unwraps: a panic)
  sg::cell_get(ri, (size_t)i * ri->n + j, latency_ns, nullptr);
  return SG_OK;
}

int32_t sg_worker_get_reliability(const sg_routing_info* ri, uint32_t src_be, uint32_t dst_be, float* reliability) {
  if (!ri || !reliability) return SG_ERR_INVALID_ARG;
  const uint32_t i = sg::row_of_ip_be(ri, src_be), j = sg::row_of_ip_be(ri, dst_be);
  if (i >= ri->n || j >= ri->n) return SG_ERR_INVALID_ARG;
  float loss;
  sg::cell_get(ri, (size_t)i * ri->n + j, nullptr, &loss);
  *reliability = 1.0f - loss;  // one f32 subtraction (worker.rs:530)
  return SG_OK;
}

int32_t sg_worker_is_routable(const sg_routing_info* ri, uint32_t src_be, uint32_t dst_be) {
  if (!ri) return 0;
  // worker.rs:544-555: both addresses resolve to a node (the graph is connected)
  return sg::row_of_ip_be(ri, src_be) != ~0u && sg::row_of_ip_be(ri, dst_be) != ~0u;
}

}  // extern "C"
