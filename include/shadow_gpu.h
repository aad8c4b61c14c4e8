/*
 * shadow_gpu.h -- C ABI of the MI355X network core for Shadow (gfx950 / HIP).
 *
 * This is the drop-in boundary for two stages of Shadow 3.2.0's network core:
 *
 *   1. Routing-table build.  Replaces
 *        NetworkGraph::compute_shortest_paths   src/main/network/graph/mod.rs:183-228
 *        NetworkGraph::get_direct_paths         src/main/network/graph/mod.rs:230-252
 *      and the id remap of generate_routing_info (src/main/core/sim_config.rs:411-448).
 *      The result is a dense table instead of HashMap<(u32,u32),PathProperties>
 *      (RoutingInfo, graph/mod.rs:434-481): row i / column j = nodes[i] / nodes[j].
 *
 *   2. Inter-host packet delivery for one scheduling round.  Replaces the
 *      per-packet body of Worker::send_packet (src/main/core/worker.rs:322-397)
 *      and WorkerShared::push_packet_to_host (worker.rs:597-607): destination
 *      resolution (Dns::addr_to_host_id, network/dns.rs:174-176), path lookup
 *      (WorkerShared::latency/reliability, worker.rs:517-531), the per-host
 *      Xoshiro256++ loss draw (host/host.rs:221,645-647), arrival time, event
 *      ids (host.rs:649-653) and the destination EventQueue order
 *      (core/work/event.rs:84-155).
 *
 * Conventions: plain C, int32_t status codes (sg_status), never unwinds.
 * Pointers documented "device" are HIP device pointers on the context's
 * device; everything else is host memory.  The reference's panics
 * (unreachable pair, graph/mod.rs:219; unit overflow, graph/mod.rs:336) become
 * status codes.  Calls on one context are not thread-safe (the reference makes
 * these calls from one thread: sim_config.rs:137 and the manager's round loop).
 */
#ifndef SHADOW_GPU_H
#define SHADOW_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG_ABI_VERSION 7

typedef enum sg_status {
  SG_OK = 0,
  SG_ERR_NO_EDGE = 1,       /* graph/mod.rs:266-268  "No edge connecting node {} to {}" */
  SG_ERR_MULTI_EDGE = 2,    /* graph/mod.rs:269-275  "More than one edge connecting node {} to {}" */
  SG_ERR_UNREACHABLE = 3,   /* graph/mod.rs:219      assert_eq!(paths.len(), n^2) (panic) */
  SG_ERR_OOM = 4,
  SG_ERR_INVALID_ARG = 5,
  SG_ERR_DEVICE = 6,        /* HIP runtime error */
  SG_ERR_PARSE = 7,         /* NetworkGraph::parse / ShadowEdge::try_from (graph/mod.rs:72-181) */
  SG_ERR_UNSORTED = 8,      /* sg_deliver_round: packets not grouped by ascending source host */
  SG_ERR_DUPLICATE_IP = 9,  /* two hosts with one address (IpAssignment::assign_ip, graph/mod.rs:383-394) */
  SG_ERR_CAPACITY = 10,     /* a CoDel queue outgrew its ring (sg_codel_create ring_cap) */
  SG_ERR_UNSUPPORTED = 12,  /* sg_comm_*: RCCL (librccl.so.1) could not be opened (ABI 7) */
  SG_ERR_TIME_OVERFLOW = 11 /* send time + latency past EMUTIME_MAX: EmulatedTime + SimulationTime
                               panics in the reference (emulated_time.rs:121-126, worker.rs:381) */
} sg_status;

typedef struct sg_ctx sg_ctx;     /* one HIP device + stream + workspace */
typedef struct sg_net sg_net;     /* device-resident network graph */
typedef struct sg_hosts sg_hosts; /* device-resident host table: addresses, routes, RNG, event ids */
typedef struct sg_gml sg_gml;     /* host-side parsed GML graph */

int32_t sg_abi_version(void);

/* ---- context ------------------------------------------------------------ */
int32_t sg_ctx_create(int32_t device, sg_ctx** out);
void sg_ctx_destroy(sg_ctx* ctx);
/* Use an existing hipStream_t (e.g. torch's current stream); NULL = the context's own
 * stream, a blocking stream (ordered with work on the legacy default stream, which is
 * torch's default stream).  Every entry point launches on this stream and reads
 * device inputs in stream order: inputs written on some other non-blocking stream
 * must be complete (or waited for) before the call. */
int32_t sg_ctx_set_stream(sg_ctx* ctx, void* hip_stream);
void* sg_ctx_stream(const sg_ctx* ctx);
int32_t sg_ctx_synchronize(sg_ctx* ctx);
/* Message and (row, col) of the last failing call on this context. */
const char* sg_ctx_last_error(const sg_ctx* ctx);
void sg_ctx_last_error_pair(const sg_ctx* ctx, uint32_t* row, uint32_t* col);
/* Measurement hooks (bench.py): with bit 0 of `enable` set, every launch of an
 * instrumented kernel is bracketed by HIP events on the context stream;
 * bit 1 (SG_TIMERS_COUNT_WORK) additionally runs the counting variant of kernels
 * whose work is data-dependent (the relaxation kernel counts the lane-
 * relaxations it performs; slower, so time and count in separate runs).
 * read_timer returns the summed device time, the launch count and the
 * algorithmic work ("relax": lane-relaxations; delivery kernels: bytes).
 * Enabling or disabling resets all timers. */
#define SG_TIMERS_ON 1
#define SG_TIMERS_COUNT_WORK 2
int32_t sg_ctx_enable_timers(sg_ctx* ctx, int32_t enable);
int32_t sg_ctx_read_timer(sg_ctx* ctx, const char* kernel, double* total_ms, uint64_t* launches,
                          double* work);

/* ---- GML ingest (NetworkGraph::parse, graph/mod.rs:134-181) -------------- */
/* Edge list in GML edge order; node indices are petgraph NodeIndex values
 * (GML node order).  Latency in integer ns (units.rs:377-438), loss f32. */
typedef struct sg_graph {
  uint32_t n_nodes;
  uint32_t n_edges;
  const uint32_t* edge_src;
  const uint32_t* edge_dst;
  const uint64_t* edge_latency_ns;
  const float* edge_packet_loss;
  const uint32_t* node_gml_id; /* optional (may be NULL): GML ids, for messages */
  uint8_t directed;
} sg_graph;

/* Parse GML text.  On failure returns SG_ERR_PARSE and writes a message into
 * err (if err_len > 0).  Latency unit overflow is reported here. */
int32_t sg_gml_parse(const char* text, size_t len, sg_gml** out, char* err, size_t err_len);
/* The same parse on `threads` host threads (0: min(cores, 16), or SG_GML_THREADS).
 * Results and the error reported are those of the single-threaded parse
 * (load_network_graph feeds it, graph/mod.rs:498-513). */
int32_t sg_gml_parse_threads(const char* text, size_t len, uint32_t threads, sg_gml** out, char* err,
                             size_t err_len);
/* load_network_graph + NetworkGraph::parse (graph/mod.rs:483-513): read the GML
 * file at `path` ("~/" expanded, tilde_expansion), xz-decompress it when
 * compression = 1 (read_xz, :484-496: the system liblzma.so.5, opened at run
 * time), check it is UTF-8 (String::from_utf8 / read_to_string), and parse it
 * on `threads` threads as sg_gml_parse_threads.  compression 0 = plain text.
 * Read, decompression and UTF-8 failures are SG_ERR_PARSE with a message. */
int32_t sg_gml_load(const char* path, uint32_t compression, uint32_t threads, sg_gml** out, char* err,
                    size_t err_len);
/* Borrow the parsed edge list (valid until sg_gml_destroy). */
int32_t sg_gml_graph(const sg_gml* g, sg_graph* out);
/* NetworkGraph::node_id_to_index (graph/mod.rs:126-128); SG_ERR_INVALID_ARG if absent. */
int32_t sg_gml_node_index(const sg_gml* g, uint32_t gml_id, uint32_t* out_index);
void sg_gml_destroy(sg_gml* g);

/* ---- routing-table build ------------------------------------------------- */
/* Upload a graph to the device and build its in-arc (CSC) form. */
int32_t sg_net_create(sg_ctx* ctx, const sg_graph* g, sg_net** out);
void sg_net_destroy(sg_net* net);

#define SG_ROUTE_SHORTEST_PATH 0x1u /* network.use_shortest_path (configuration.rs:315-326) */
#define SG_ROUTE_OUT_DEVICE 0x2u    /* out_* are device pointers (else host) */

/*
 * Rows [row_begin, row_end) of the routing table over `nodes` (petgraph
 * indices of the used nodes, n_used of them; the caller's order defines the
 * table's row/column order):
 *   out_latency_ns [(i-row_begin)*n_used + j] = path(nodes[i] -> nodes[j]).latency_ns
 *   out_packet_loss[(i-row_begin)*n_used + j] = path(nodes[i] -> nodes[j]).packet_loss
 * With SG_ROUTE_SHORTEST_PATH: the lexicographic (latency, loss) optimum of
 * the left fold PathProperties::default() + e1 + ... + ek over every path,
 * bit-exact (petgraph::algo::dijkstra semantics), diagonal = the node's single
 * self-loop.  Without: the single direct edge of every pair.
 * Errors as the reference: missing/duplicate self-loop (first node in order),
 * missing/duplicate direct edge (first pair in row-major order), unreachable
 * pair (first pair in row-major order); sg_ctx_last_error_pair gives (i, j).
 * Rows may be sharded across devices by calling with disjoint row ranges.
 */
int32_t sg_routing_build(sg_ctx* ctx, sg_net* net, const uint32_t* nodes, uint32_t n_used,
                         uint32_t row_begin, uint32_t row_end, uint32_t flags,
                         uint64_t* out_latency_ns, float* out_packet_loss);

/* RoutingInfo::get_smallest_latency_ns (graph/mod.rs:478-480) over `count`
 * device latencies; UINT64_MAX when count == 0. */
int32_t sg_routing_min_latency(sg_ctx* ctx, const uint64_t* d_latency_ns, size_t count,
                               uint64_t* out_min);

/* ---- host-side dense RoutingInfo (graph/mod.rs:432-481) ------------------
 * RoutingInfo<u32> keyed by GML node id, as generate_routing_info builds it
 * (sim_config.rs:411-448), stored dense: row-major latency / loss arrays in
 * pinned host memory owned by the object and an id -> row map.  It replaces the
 * reference's two n_used^2 HashMaps (compute_shortest_paths', graph/mod.rs:190-208,
 * and the id remap's, sim_config.rs:423-445) and answers RoutingInfo::path and
 * the WorkerShared lookups with array reads.  Lookups are read-only and safe
 * from any number of threads; packet counters are atomic.                    */
typedef struct sg_routing_info sg_routing_info;
/* node_ids: the used GML node ids (the table's row / column order).  Allocates
 * the n_used^2 table of 8-byte cells (pinned when a HIP device is present).  SG_ERR_INVALID_ARG
 * for a duplicate id. */
int32_t sg_routing_info_create(uint32_t n_used, const uint32_t* node_ids, sg_routing_info** out);
void sg_routing_info_destroy(sg_routing_info* ri);
/* Build the whole table: nodes[i] = the petgraph index of node_ids[i]
 * (NetworkGraph::node_id_to_index, graph/mod.rs:126-128).  Results and errors
 * are sg_routing_build's over all rows; row blocks are built on the device and
 * copied into the object while the next block builds.  Also computes
 * get_smallest_latency_ns. */
int32_t sg_routing_info_fill(sg_ctx* ctx, sg_net* net, const uint32_t* nodes, uint32_t flags, sg_routing_info* ri);
/* Rows [row_begin, row_end) from host arrays (e.g. row shards gathered from
 * other ranks' sg_routing_build).  get_smallest_latency_ns is Some once every row
 * has been set (by fill or by these calls), over the whole table. */
int32_t sg_routing_info_set_rows(sg_routing_info* ri, uint32_t row_begin, uint32_t row_end,
                                 const uint64_t* latency_ns, const float* packet_loss);
/* Zero-copy view: cell (i, j) = path(node_ids[i] -> node_ids[j]) packed as
 * (latency_ns << 32) | bits(packet_loss), 8 bytes, while the latency is below
 * SG_CELL_WIDE; a cell whose upper half is SG_CELL_WIDE holds its loss bits only,
 * and its u64 latency is one of the n_wide entries that sg_routing_info_rows and
 * the lookups below resolve (paths of 4.29 s or more are rare: the whole table
 * moves and lives at 8 bytes per cell instead of 12). */
#define SG_CELL_WIDE 0xFFFFFFFFu
typedef struct sg_routing_view {
  uint32_t n;
  const uint32_t* node_ids;
  const uint64_t* cells;
  uint64_t n_wide;
  uint32_t pinned;
} sg_routing_view;
int32_t sg_routing_info_view(const sg_routing_info* ri, sg_routing_view* out);
/* Rows [row_begin, row_end) decoded into caller arrays (latency u64, loss f32, row-major). */
int32_t sg_routing_info_rows(const sg_routing_info* ri, uint32_t row_begin, uint32_t row_end, uint64_t* latency_ns,
                             float* packet_loss);
/* Row of a GML node id (SG_ERR_INVALID_ARG if absent). */
int32_t sg_routing_info_index(const sg_routing_info* ri, uint32_t node_id, uint32_t* row);
/* RoutingInfo::path(start, end) (graph/mod.rs:448-450): 1 = Some (outputs
 * written when non-NULL), 0 = None. */
int32_t sg_routing_info_path(const sg_routing_info* ri, uint32_t start, uint32_t end, uint64_t* latency_ns,
                             float* packet_loss);
/* RoutingInfo::get_smallest_latency_ns (graph/mod.rs:478-480): 1 = Some, 0 = None. */
int32_t sg_routing_info_smallest_latency(const sg_routing_info* ri, uint64_t* out);
/* RoutingInfo::increment_packet_count (graph/mod.rs:453-460): saturating, thread
 * safe; SG_ERR_INVALID_ARG for an unknown pair (its caller unwraps, worker.rs:538-542). */
int32_t sg_routing_info_increment_packet_count(sg_routing_info* ri, uint32_t start, uint32_t end);
uint64_t sg_routing_info_packet_count(const sg_routing_info* ri, uint32_t start, uint32_t end);
/* IpAssignment (graph/mod.rs:354-430): the assigned addresses (host byte order,
 * u32::from(Ipv4Addr)) and their GML node ids; SG_ERR_DUPLICATE_IP for a repeat. */
int32_t sg_routing_info_set_addresses(sg_routing_info* ri, uint32_t n_addrs, const uint32_t* ipv4,
                                      const uint32_t* node_id);
/* WorkerShared::latency / reliability / is_routable (worker.rs:517-555) as the C
 * exports worker_getLatency / worker_isRoutable take them (worker.rs:651-684):
 * addresses in network byte order.  latency / reliability return SG_OK, or
 * SG_ERR_INVALID_ARG where the reference's Option is None (worker_getLatency
 * unwraps it: a panic).  reliability = 1f32 - loss.  is_routable: 1 when both
 * addresses are assigned (the graph is connected), else 0. */
int32_t sg_worker_get_latency(const sg_routing_info* ri, uint32_t src_be, uint32_t dst_be, uint64_t* latency_ns);
int32_t sg_worker_get_reliability(const sg_routing_info* ri, uint32_t src_be, uint32_t dst_be, float* reliability);
int32_t sg_worker_is_routable(const sg_routing_info* ri, uint32_t src_be, uint32_t dst_be);

/* ---- packet delivery ------------------------------------------------------ */
/*
 * Host table.  host_ipv4[h] = the host's address (host byte order, as
 * u32::from(Ipv4Addr)); host_route_idx[h] = index of the host's graph node in
 * the routing table's node list; host_seed[h] = HostInfo.seed (node_seed):
 * the RNG is Xoshiro256PlusPlus::seed_from_u64(seed) (host.rs:221).  HostId =
 * h (hosts sorted by name, configuration.rs:107).  Addresses must be unique.
 */
int32_t sg_hosts_create(sg_ctx* ctx, uint32_t n_hosts, const uint32_t* host_ipv4,
                        const uint32_t* host_route_idx, const uint64_t* host_seed,
                        sg_hosts** out);
/* Copy RNG state (4 u64 per host, Xoshiro s[0..3]) and event-id counters
 * (Host::event_id_counter) out of / into the device (host memory). */
int32_t sg_hosts_get_state(sg_hosts* hosts, uint64_t* rng_state, uint64_t* event_ctr);
int32_t sg_hosts_set_state(sg_hosts* hosts, const uint64_t* rng_state, const uint64_t* event_ctr);
/* Advance hosts' device RNG streams by steps[i] next_u64 steps each (host
 * arrays, n entries, host_ids[i] < n_hosts; a host may repeat): the steps other
 * consumers took (see sg_packets.rng_skip) that no later packet has carried to
 * the device yet -- e.g. before sg_hosts_get_state for a checkpoint. */
int32_t sg_hosts_skip(sg_hosts* hosts, uint32_t n, const uint32_t* host_ids, const uint64_t* steps);
void sg_hosts_destroy(sg_hosts* hosts);

/* Routing-table shard resident on the device (rows [row_begin, row_begin+n_rows)).
 * path_key (optional, from sg_table_pack) holds each cell as one u64,
 * (latency_ns << 32) | bits(packet_loss): the delivery walk then gathers one
 * 8-byte word per packet instead of two scattered words.  When path_key is
 * set, latency_ns / packet_loss are not read by the delivery calls and may be
 * NULL.  NULL = use the two arrays. */
typedef struct sg_table {
  const uint64_t* latency_ns; /* device, n_rows x n_cols */
  const float* packet_loss;   /* device, n_rows x n_cols */
  uint32_t n_cols;
  uint32_t row_begin;
  uint32_t n_rows;
  const uint64_t* path_key;   /* device, n_rows x n_cols, or NULL */
} sg_table;

/* ABI 7: per-pair packet counters on the device.  RoutingInfo::increment_packet_count
 * (graph/mod.rs:451-459), which Worker::send_packet calls for every delivered
 * packet (worker.rs:373): with counters set, every sg_deliver_round /
 * sg_deliver_source on this context adds one to counts[cell] for each packet it
 * delivers, cell = the path's cell of the table it was given ((route row -
 * row_begin) * n_cols + destination column).  counts: device u64, n_cells >=
 * the table's n_rows * n_cols, zeroed by the caller (the reference's counters
 * start empty); NULL turns counting off (the default).  The reference
 * saturates its u64; a u64 count of packets cannot reach it. */
int32_t sg_ctx_set_packet_counters(sg_ctx* ctx, uint64_t* counts, uint64_t n_cells);

/* Pack a table's (latency_ns, packet_loss) cells into path_key form
 * (out_key: device, n_rows x n_cols u64).  *out_packable (host) = 1 if every
 * latency is below 2^32 ns, else 0 and out_key must not be used (latencies of
 * 4.29 s and more keep the two-array form).  Synchronises.  Done once per
 * routing table (the table is immutable for the simulation, network_graph.rs
 * IpPreviewTable / RoutingInfo are built once in Manager::run). */
int32_t sg_table_pack(sg_ctx* ctx, const sg_table* table, uint64_t* out_key, uint32_t* out_packable);

/* Round clock (EmulatedTime ns).  round_end = the worker's barrier
 * (worker.rs:262-268); sim_end / bootstrap_end from WorkerShared. */
typedef struct sg_round {
  uint64_t round_end_ns;
  uint64_t sim_end_ns;
  uint64_t bootstrap_end_ns;
} sg_round;

/* One round's sent packets, device SoA, grouped by ascending source host and
 * in each host's send order (the order Worker::send_packet saw them).
 *
 * rng_skip (optional, NULL = none): the host's Xoshiro stream is shared with
 * other consumers on the CPU -- Host::random_mut() (host.rs:645-647) is also
 * drawn by getrandom (syscall/handler/random.rs:40), socket port choices
 * (socket.rs:179-858), host_rngDouble / host_rngNextNBytes (host.rs:1288-1300)
 * and the auxv random bytes (managed_thread.rs:248).  rng_skip[i] = the number
 * of next_u64 steps those consumers took on packet i's source host since the
 * previous packet of that host handed to the device (in this batch or an
 * earlier one).  The device advances the host's stream by that many steps
 * before packet i (whatever its status), so every packet draws at exactly the
 * stream position Worker::send_packet (worker.rs:360) drew from.  The CPU keeps
 * its own copy of the stream in step by taking one step per packet that draws
 * (now < sim_end and the destination resolves, worker.rs:332-360): no state
 * crosses the bus per round. */
typedef struct sg_packets {
  uint32_t n_packets;
  const uint32_t* src_host;     /* HostId of the sending host */
  const uint32_t* dst_ipv4;     /* destination address (host byte order) */
  const uint32_t* payload_len;  /* PacketRc::payload_len (packet.rs:394-396) */
  const uint64_t* send_time_ns; /* Worker::current_time() at the send */
  const uint32_t* rng_skip;     /* device, n_packets, or NULL (see above) */
} sg_packets;

enum {
  SG_PKT_DELIVERED = 0,  /* PacketStatus::InetSent; pushed to the destination queue */
  SG_PKT_DROP_LOSS = 1,  /* InetDropped by the reliability draw (worker.rs:365-368) */
  SG_PKT_DROP_NO_DST = 2,/* InetDropped: unknown destination, no draw (worker.rs:341-351) */
  SG_PKT_SIM_END = 3     /* now >= sim_end: ignored, no draw (worker.rs:332-335) */
};

/* Device outputs. */
typedef struct sg_deliveries {
  uint8_t* status;           /* n_packets, SG_PKT_* */
  uint64_t* deliver_time_ns; /* n_packets (0 unless delivered) */
  uint64_t* event_id;        /* n_packets, src_host_event_id (UINT64_MAX unless delivered) */
  uint32_t* dst_order;       /* n_packets capacity: delivered packet indices bucketed by
                                destination, each bucket in EventQueue pop order */
  uint32_t* dst_offsets;     /* n_hosts + 1 */
} sg_deliveries;

typedef struct sg_round_stats {
  uint64_t n_delivered;
  uint64_t min_deliver_time_ns; /* Worker::update_next_event_time input min (worker.rs:388) */
  uint64_t min_used_latency_ns; /* Worker::update_lowest_used_latency input min (worker.rs:372) */
} sg_round_stats;

/* Run one round.  Updates the hosts' RNG streams and event counters on the
 * device.  `stats` (host) may be NULL for a fully asynchronous call.
 * A batch that is not grouped by ascending source host (SG_ERR_UNSORTED), names
 * a host out of range, or comes from a host whose route row is outside the
 * table shard (SG_ERR_INVALID_ARG) is rejected whole: no host's RNG stream or
 * event counter changes and no output is written.  SG_ERR_TIME_OVERFLOW (the
 * reference panics) leaves the hosts' state undefined. */
int32_t sg_deliver_round(sg_ctx* ctx, sg_hosts* hosts, const sg_table* table,
                         const sg_round* round, const sg_packets* packets, sg_deliveries* out,
                         sg_round_stats* stats);

/* ---- sharded delivery (one process per GPU, exchange between the calls) ---
 * Hosts are partitioned over ranks; a rank sends for the hosts whose routing
 * rows it holds and receives for the hosts it owns.
 *   1. sg_deliver_source: the send_packet half for this rank's packets
 *      (same per-packet outputs and RNG/counter updates as sg_deliver_round),
 *      plus one sg_record per delivered packet, grouped by the destination's
 *      owner rank host_owner[dst] (send_counts[r] records for rank r, in rank
 *      order).  Synchronises (the counts are needed for the exchange).
 *   2. the caller exchanges records (all-to-all, e.g. RCCL over xGMI).
 *   3. sg_deliver_bucket: the push_packet_to_host half on the owner: bucket
 *      the received records by local destination slot host_local[dst] and
 *      order each bucket as the EventQueue pops it (deliver time, src host,
 *      event id).  dst_order holds indices into `recv`.                     */
typedef struct sg_record {
  uint64_t deliver_time_ns;
  uint64_t order_key; /* (src_host << 32) | k, k = rank among src_host's delivered packets this round */
  uint64_t event_id;  /* src_host_event_id */
  uint32_t packet;    /* index in the source rank's sg_packets */
  uint32_t dst_host;  /* HostId of the destination */
} sg_record;

int32_t sg_deliver_source(sg_ctx* ctx, sg_hosts* hosts, const sg_table* table, const sg_round* round,
                          const sg_packets* packets, uint8_t* status, uint64_t* deliver_time_ns,
                          uint64_t* event_id, const uint32_t* host_owner, uint32_t n_ranks,
                          sg_record* send, uint32_t* send_counts, sg_round_stats* stats);
int32_t sg_deliver_bucket(sg_ctx* ctx, const sg_record* recv, uint32_t n_records,
                          const uint32_t* host_local, uint32_t n_hosts, uint32_t n_local_hosts,
                          uint32_t* dst_order, uint32_t* dst_offsets);

/* ---- sharded delivery with a fixed-split exchange (no host round trip) ----
 * The same round as sg_deliver_source / sg_deliver_bucket, with every rank's
 * records for rank r in a block of `cap` slots, so the exchange is one
 * equal-split all-to-all the host need not size (RCCL over xGMI), and the round
 * synchronises once, at its end.  `cap` must be the same on every rank (e.g.
 * derived from the largest pair count of the round before).
 *   1. sg_deliver_source_padded: the source half; rank r's k-th record goes to
 *      send_padded[r * cap + k] if k < cap, else to its compact position in
 *      `send` (n_packets records, as sg_deliver_source's).  xrow (device,
 *      3 + n_ranks u64) = [delivered, min deliver time, min used latency,
 *      records for rank 0, 1, ...].  Does not synchronise.
 *   2. the caller all-gathers xrow into xall (n_ranks x (3 + n_ranks)) and
 *      all-to-alls send_padded (cap records per rank pair) into recv_padded.
 *   3. sg_deliver_bucket_padded: buckets the valid records of every block (block
 *      b holds min(xall[b][3 + rank], cap)); dst_order indexes recv_padded.
 *      stats = the round's global values; recv_counts[b] = records rank b sent
 *      this rank; pair_max = the largest count any rank sent any rank.  If
 *      pair_max > cap, some records did not fit: every rank sees the same xall,
 *      so all of them then run sg_deliver_pad_to_compact (the complete compact
 *      `send`), the exact exchange of sg_deliver_source's protocol with the
 *      counts from xall, and sg_deliver_bucket.                                */
int32_t sg_deliver_source_padded(sg_ctx* ctx, sg_hosts* hosts, const sg_table* table, const sg_round* round,
                                 const sg_packets* packets, uint8_t* status, uint64_t* deliver_time_ns,
                                 uint64_t* event_id, const uint32_t* host_owner, uint32_t n_ranks, uint32_t cap,
                                 sg_record* send_padded, sg_record* send, uint64_t* xrow);
int32_t sg_deliver_bucket_padded(sg_ctx* ctx, const sg_record* recv_padded, uint32_t n_ranks, uint32_t cap,
                                 const uint64_t* xall, uint32_t rank, const uint32_t* host_local, uint32_t n_hosts,
                                 uint32_t n_local_hosts, uint32_t* dst_order, uint32_t* dst_offsets,
                                 sg_round_stats* stats, uint32_t* recv_counts, uint32_t* pair_max);
int32_t sg_deliver_pad_to_compact(sg_ctx* ctx, const sg_record* send_padded, uint32_t n_ranks, uint32_t cap,
                                  const uint64_t* xrow, sg_record* send);

/* ---- collectives of the sharded path over RCCL (ABI 7) --------------------
 * One communicator per rank (one process per GPU), bound to an sg_ctx: every call
 * is enqueued on the context's stream, after the library's kernels, and returns
 * without synchronising.  They replace the hand-offs between the reference's
 * worker threads (Worker::push_packet_to_host, worker.rs:597-607, run from the
 * manager's round loop, manager.rs:415-501) and the routing table every worker
 * reads (NetworkGraph::compute_shortest_paths, graph/mod.rs:183-228, computed once,
 * sim_config.rs:137-141) once rows and hosts are sharded over GPUs.  RCCL is
 * opened at run time (librccl.so.1); without it these return SG_ERR_UNSUPPORTED
 * and everything else works.
 *   sg_comm_unique_id: on one rank; the caller passes the bytes to every rank.
 *   sg_comm_allgather_rows: in place, rank r's rows [r rows_per_rank, (r + 1)
 *     rows_per_rank) of the n_used-column table (device lat u64 / loss f32; either
 *     may be NULL) to every rank.
 *   sg_comm_exchange_padded: step 2 of the fixed-split round above: xrow (3 +
 *     n_ranks u64, device) all-gathered into xall, and cap records per rank pair
 *     from send_padded to recv_padded (n_ranks blocks each).
 *   sg_comm_alltoallv_records: the exact exchange of sg_deliver_source's records
 *     (grouped by rank: send_counts[r] for rank r), received rank after rank;
 *     send_counts / recv_counts are host arrays of n_ranks.
 *   sg_comm_allgather_u64: n u64 per rank (device) into all (n_ranks x n).   */
typedef struct sg_comm sg_comm;
#define SG_COMM_ID_BYTES 128
int32_t sg_comm_unique_id(uint8_t* id /* SG_COMM_ID_BYTES */);
int32_t sg_comm_create(sg_ctx* ctx, const uint8_t* id, uint32_t n_ranks, uint32_t rank, sg_comm** out);
void sg_comm_destroy(sg_comm* comm);
int32_t sg_comm_allgather_rows(sg_comm* comm, uint64_t* lat, float* loss, uint32_t rows_per_rank, uint32_t n_used);
int32_t sg_comm_exchange_padded(sg_comm* comm, const sg_record* send_padded, sg_record* recv_padded, uint32_t cap,
                                const uint64_t* xrow, uint64_t* xall);
int32_t sg_comm_alltoallv_records(sg_comm* comm, const sg_record* send, const uint32_t* send_counts,
                                  sg_record* recv, const uint32_t* recv_counts);
int32_t sg_comm_allgather_u64(sg_comm* comm, const uint64_t* mine, uint64_t* all, uint32_t n);

/* ---- router inbound CoDel queues (one per host) ---------------------------
 * Router::inbound_packets (router/mod.rs:15-58): each host's CoDelQueue
 * (router/codel_queue.rs), RFC 8289 with Shadow's TARGET = 10 ms,
 * INTERVAL = 100 ms, no LIMIT, MTU = 1500 (definitions.h:124).  The queues
 * and their CoDel state live on the device across calls.  A call runs a batch
 * of push / pop events: each host's events in its order (hosts are
 * independent, so the batch runs one device lane per host).
 *   push(packet, len, now)  = CoDelQueue::push (codel_queue.rs:303-317)
 *   pop(now) -> packet|none = CoDelQueue::pop  (codel_queue.rs:125-148),
 *                             dropping as the control law dictates.      */
typedef struct sg_codel sg_codel;
enum { SG_CODEL_PUSH = 0, SG_CODEL_POP = 1 };
enum { SG_CODEL_QUEUED = 0, SG_CODEL_DEQUEUED = 1, SG_CODEL_DROPPED = 2 /* PacketStatus::RouterDropped */ };

/* ring_cap: packets a host's queue may hold (rounded up to a power of two);
 * a push beyond it fails the call with SG_ERR_CAPACITY (the reference has no
 * limit, so size it for the workload). */
int32_t sg_codel_create(sg_ctx* ctx, uint32_t n_hosts, uint32_t ring_cap, sg_codel** out);
void sg_codel_destroy(sg_codel* q);

typedef struct sg_codel_events { /* device arrays, grouped by ascending host */
  uint32_t n_events;
  const uint32_t* host;
  const uint8_t* kind;     /* SG_CODEL_PUSH | SG_CODEL_POP */
  const uint64_t* time_ns; /* EmulatedTime of the operation (Worker::current_time) */
  const uint32_t* packet;  /* push: the caller's packet id (< n_packets below) */
  const uint32_t* len;     /* push: PacketRc::len() (packet.rs:388-390) */
} sg_codel_events;

/* pop_result (device, n_events): the popped packet id, UINT32_MAX for an
 * empty pop and for pushes.  pkt_status (device, n_packets): set to
 * SG_CODEL_DEQUEUED / SG_CODEL_DROPPED when a packet leaves its queue.
 * n_dropped (host, may be NULL): packets CoDel dropped in this call. */
int32_t sg_codel_run(sg_ctx* ctx, sg_codel* q, const sg_codel_events* ev, uint32_t* pop_result,
                     uint8_t* pkt_status, uint32_t n_packets, uint64_t* n_dropped);

/* Copy the per-host state out of / into the device (host arrays, n_hosts
 * each; ring_* n_hosts * ring_cap): flags (bit 0 drop mode, bit 1
 * interval_end set, bit 2 drop_next set), interval_end, drop_next, current /
 * previous drop count, bytes stored, ring head / tail counters, and the ring
 * (packet, enqueue time, len).  For checkpoints and tests. */
typedef struct sg_codel_state {
  uint8_t* flags;
  uint64_t *interval_end, *drop_next, *cur_drops, *prev_drops, *bytes;
  uint32_t *head, *tail;
  uint32_t* ring_packet;
  uint64_t* ring_time;
  uint32_t* ring_len;
} sg_codel_state;
uint32_t sg_codel_ring_cap(const sg_codel* q);
int32_t sg_codel_get_state(sg_codel* q, sg_codel_state* out);
int32_t sg_codel_set_state(sg_codel* q, const sg_codel_state* in);

/* ---- inbound pipeline: router CoDel queue -> relay_inet_in (token bucket) --
 * Host::execute on a Packet event (host.rs:781-786): the packet enters the
 * router's CoDel queue and the inbound relay is notified; the relay
 * (relay/mod.rs:72-288) forwards from the queue to the host's internet
 * interface as its token bucket allows (relay/token_bucket.rs: refill
 * max(1, bw_down_bytes / 1000) every 1 ms, capacity refill + MTU,
 * relay/mod.rs:296-309), rescheduling itself when blocked.  A call processes
 * one host's arrivals (a delivery round's buckets, in EventQueue order) and the
 * relay's forward tasks up to window_end; later tasks stay pending.  Assumes
 * Shadow's CPU-delay model is off (host.rs:758-775; its default).           */
typedef struct sg_inbound sg_inbound;
/* bw_down_bits (host, n_hosts): each host's bandwidth down (HostInfo, bits/s). */
int32_t sg_inbound_create(sg_ctx* ctx, uint32_t n_hosts, const uint64_t* bw_down_bits, uint32_t ring_cap,
                          sg_inbound** out);
void sg_inbound_destroy(sg_inbound* ib);
uint32_t sg_inbound_ring_cap(const sg_inbound* ib);

typedef struct sg_inbound_arrivals { /* device arrays, grouped by ascending host, EventQueue order */
  uint32_t n;
  const uint32_t* host;
  const uint64_t* time_ns; /* the Packet event's time (the delivery's arrival), < window_end */
  const uint32_t* packet;  /* the caller's packet id (< n_packets) */
  const uint32_t* len;     /* PacketRc::len() */
} sg_inbound_arrivals;

/* Packet ids are below n_packets <= 2^31: SG_ERR_INVALID_ARG otherwise, for an id at or past
 * n_packets as soon as it enters a queue (sg_inbound_run) or would stay queued past the call
 * (sg_inbound_run_ordered).
 * event_ctr (device, n_hosts, may be NULL): each host's event-id counter,
 * advanced by one per forward task the relay schedules (host.rs:649-653) --
 * e.g. sg_hosts_event_ctr(hosts).  fwd_time (device, n_packets): the time the
 * relay pushed the packet to the interface; pkt_status (device, n_packets):
 * SG_CODEL_DEQUEUED once forwarded, SG_CODEL_DROPPED if CoDel dropped it.
 * n_dropped (host, may be NULL): CoDel drops in this call. */
int32_t sg_inbound_run(sg_ctx* ctx, sg_inbound* ib, const sg_inbound_arrivals* arr, uint64_t window_end_ns,
                       uint64_t bootstrap_end_ns, uint64_t sim_end_ns, uint64_t* event_ctr, uint64_t* fwd_time,
                       uint8_t* pkt_status, uint32_t n_packets, uint64_t* n_dropped);

/* ABI 7: the same call with each arrival's fate written in arrival order
 * (RelayForwarded / drop_packet of relay/mod.rs:201-273 and
 * codel_queue.rs:125-148, at the arrival's index instead of its packet id, so
 * a host's outputs are consecutive).  arr_status (device, arr->n): set to
 * SG_CODEL_DEQUEUED / SG_CODEL_DROPPED when arrival i of this call leaves its
 * queue in this call, untouched while it stays queued (the caller zeroes it:
 * SG_CODEL_QUEUED); arr_fwd_time (device, arr->n): the forward time of a
 * DEQUEUED arrival, untouched otherwise.  Packets that arrived in earlier calls
 * and leave in this one still go to pkt_status / fwd_time by packet id
 * (n_packets covers every id).  arr->n < 2^31. */
int32_t sg_inbound_run_ordered(sg_ctx* ctx, sg_inbound* ib, const sg_inbound_arrivals* arr, uint64_t window_end_ns,
                               uint64_t bootstrap_end_ns, uint64_t sim_end_ns, uint64_t* event_ctr,
                               uint64_t* fwd_time, uint8_t* pkt_status, uint32_t n_packets, uint64_t* arr_fwd_time,
                               uint8_t* arr_status, uint64_t* n_dropped);

typedef struct sg_inbound_relay_state { /* host arrays, n_hosts each */
  uint8_t* flags;          /* bit 0 a forward task is pending, bit 1 it was never queued (>= sim_end),
                              bit 2 a packet is cached (RelayCached) */
  uint64_t* task_time;
  uint32_t *cached_packet, *cached_len;
  uint64_t *tb_capacity, *tb_balance, *tb_increment, *tb_last_refill;
  /* ABI 6 (may be NULL): the pending forward task's Local event id
     (Host::get_new_event_id, host.rs:649-653, taken from event_ctr when the
     task was scheduled) and the time it was scheduled at (its creation). */
  uint64_t *task_event_id, *task_created_ns;
} sg_inbound_relay_state;
int32_t sg_inbound_get_state(sg_inbound* ib, sg_codel_state* queue, sg_inbound_relay_state* relay);

/* ---- outbound pipeline: network interface -> relay_inet_out -> router ------
 * The send side of the relay.  A socket with data joins
 * its interface's sending queue and relay_inet_out is notified
 * (Host::notify_socket_has_packets, host.rs:930-945; interface.rs:168-182).
 * Under the default fifo qdisc the interface pops the socket whose next packet
 * has the smallest priority (interface.rs:225-260, queuing.rs:16-36), so
 * packets leave in creation order: a host's sends are one FIFO.  The relay
 * (relay/mod.rs:111-275) pops and forwards while its token bucket allows
 * (bw_up: refill max(1, bw_up_bytes / 1000) every 1 ms, capacity refill + MTU,
 * relay/mod.rs:278-319; no limit while bootstrapping).  A packet addressed to
 * the host's own address goes back to the interface without using tokens
 * (is_local, :222-226, :259-264); any other one goes to the router, whose push
 * is Worker::send_packet at the forward task's time (router/mod.rs:41-43).
 * Those packets form an sg_packets batch for sg_deliver_round.
 *
 * A call processes each host's sends (times < window_end, nondecreasing per
 * host) and the relay's forward tasks before window_end; later tasks stay
 * pending.  Assumes Shadow's CPU-delay model is off (host.rs:758-775; its
 * default).
 *
 * Same-time order.  A send happens while the host runs some event E; the
 * relay's forward task is a Local event (relay/mod.rs:145-157).  At one
 * EmulatedTime the host runs Packet events first, then Local events by event
 * id (event.rs:84-155, :163-183), and ids grow in creation order
 * (host.rs:649-653).  With sends->event_id given, a task at time t runs before
 * a send at t iff E is a Local event created after the task:
 * (event_created_ns, event_id) > (task created, task id), the task's id taken
 * from event_ctr when it is scheduled.  event_id = UINT64_MAX marks E as a
 * Packet event (it precedes every Local one).  Creation time decides first
 * because ids are monotone in creation order, so the comparison is exact
 * whenever the two were created at different times, whatever numbering the
 * caller's own ids use within a window; at one creation time it falls back
 * to the ids.  Without event_id (NULL) every send at t
 * precedes a task at t (all sends treated as Packet-event sends).          */
typedef struct sg_outbound sg_outbound;
/* host_ipv4, bw_up_bits (host, n_hosts): each host's address and bandwidth up
 * (HostInfo, bits/s).  ring_cap bounds, per host and call, the packets queued
 * at the start (a cached one included) plus the call's sends; more fails the
 * call with SG_ERR_CAPACITY. */
int32_t sg_outbound_create(sg_ctx* ctx, uint32_t n_hosts, const uint32_t* host_ipv4, const uint64_t* bw_up_bits,
                           uint32_t ring_cap, sg_outbound** out);
void sg_outbound_destroy(sg_outbound* ob);
uint32_t sg_outbound_ring_cap(const sg_outbound* ob);

typedef struct sg_outbound_sends { /* device arrays, grouped by ascending host, interface order */
  uint32_t n;
  const uint32_t* host;
  const uint64_t* time_ns;      /* when the socket handed the packet to the interface, < window_end */
  const uint32_t* packet;       /* the caller's packet id (< n_packets) */
  const uint32_t* len;          /* PacketRc::len() (packet.rs:388-390): the bucket's cost */
  const uint32_t* payload_len;  /* PacketRc::payload_len(): carried into the sent batch */
  const uint32_t* dst_ipv4;
  /* ABI 6, optional (NULL, or both): the sending event's id and the time it was
     created (scheduled).  event_id UINT64_MAX: a Packet event.  Sends at one time
     come in the host's execution order: Packet-event sends first, then by
     (event_created_ns, event_id).  Requires event_ctr in sg_outbound_run. */
  const uint64_t* event_id;
  const uint64_t* event_created_ns;
} sg_outbound_sends;

enum { SG_OUT_QUEUED = 0, SG_OUT_SENT = 1 /* to the router: Worker::send_packet */,
       SG_OUT_LOCAL = 2 /* dst == own address: back to the interface */ };

/* The packets this call handed to send_packet, device arrays of capacity
 * `cap`, grouped by ascending host and in each host's send order: the
 * sg_packets of a delivery round (src_host, dst_ipv4, payload_len,
 * send_time_ns), plus the caller's packet id. */
typedef struct sg_outbound_sent {
  uint32_t cap;
  uint32_t *src_host, *dst_ipv4, *payload_len;
  uint64_t* send_time_ns;
  uint32_t* packet;
} sg_outbound_sent;

/* event_ctr (device, n_hosts, may be NULL): advanced by one per forward task
 * scheduled (host.rs:649-653).  fwd_time / pkt_status (device, n_packets): the
 * forward time and SG_OUT_SENT / SG_OUT_LOCAL of each packet the relay
 * forwarded (untouched otherwise).  sent may be NULL; n_sent (host, may be
 * NULL) receives the count.  SG_ERR_CAPACITY if sent->cap is too small. */
int32_t sg_outbound_run(sg_ctx* ctx, sg_outbound* ob, const sg_outbound_sends* sends, uint64_t window_end_ns,
                        uint64_t bootstrap_end_ns, uint64_t sim_end_ns, uint64_t* event_ctr, uint64_t* fwd_time,
                        uint8_t* pkt_status, uint32_t n_packets, sg_outbound_sent* sent, uint32_t* n_sent);

/* Host arrays: per host the ring head / tail counters and n_hosts * ring_cap
 * slots (packet, len, payload_len, dst).  A cached packet (relay flags bit 2)
 * is the slot at head - 1. */
typedef struct sg_outbound_queue_state {
  uint32_t *head, *tail;
  uint32_t *ring_packet, *ring_len, *ring_payload_len, *ring_dst;
} sg_outbound_queue_state;
int32_t sg_outbound_get_state(sg_outbound* ob, sg_outbound_queue_state* queue, sg_inbound_relay_state* relay);

/* The device array of the hosts' event-id counters (Host::event_id_counter). */
uint64_t* sg_hosts_event_ctr(sg_hosts* hosts);

#ifdef __cplusplus
}
#endif
#endif /* SHADOW_GPU_H */
