//! Raw bindings to `libshadow_gpu.so`, the MI355X network core for Shadow 3.2.0.
//!
//! Every declaration mirrors `include/shadow_gpu.h` (ABI 7) one to one: the 73 entry
//! points, the 15 `#[repr(C)]` structs, the opaque handles and the constants.
//! `tests/test_rust_binding_cpu.py` parses both files and fails on any difference in
//! names, argument counts, argument and field types, or constant values, and on any
//! export of the built library that this file does not declare.
//!
//! Conventions (as the header's): every fallible call returns an `i32` status
//! (`SG_OK` or `SG_ERR_*`, never unwinds); pointers the header documents as "device"
//! are HIP device pointers on the context's device, everything else is host memory.
//! The safe wrappers Shadow would use (`src/main/network/gpu.rs` in INTEGRATION.md)
//! sit on top of these and keep the reference's own types at their call sites:
//! `NetworkGraph` (`src/main/network/graph/mod.rs:116-252`), `RoutingInfo`
//! (`graph/mod.rs:432-481`), `Worker::send_packet` (`src/main/core/worker.rs:322-397`)
//! and the exported `worker_getLatency` / `worker_isRoutable`
//! (`worker.rs:619-684`, whose `extern "C-unwind"` conventions these follow in reverse:
//! plain integers and pointers, no Rust types across the boundary).
#![allow(non_camel_case_types)]
#![no_std]

use core::ffi::{c_char, c_void};

// ---------------------------------------------------------------------------
// Opaque handles
// ---------------------------------------------------------------------------
/// One HIP device, stream and workspace.
#[repr(C)]
pub struct sg_ctx {
    _private: [u8; 0],
}
/// A device-resident network graph (the petgraph `Graph` of `NetworkGraph`, graph/mod.rs:116-119).
#[repr(C)]
pub struct sg_net {
    _private: [u8; 0],
}
/// Device-resident host table: addresses, routes, Xoshiro streams, event-id counters.
#[repr(C)]
pub struct sg_hosts {
    _private: [u8; 0],
}
/// A host-side parsed GML graph (`NetworkGraph::parse`, graph/mod.rs:134-181).
#[repr(C)]
pub struct sg_gml {
    _private: [u8; 0],
}
/// The dense host-side `RoutingInfo<u32>` (graph/mod.rs:432-481).
#[repr(C)]
pub struct sg_routing_info {
    _private: [u8; 0],
}
/// One RCCL communicator bound to an `sg_ctx` (ABI 7).
#[repr(C)]
pub struct sg_comm {
    _private: [u8; 0],
}
/// Every host's router `CoDelQueue` (router/codel_queue.rs).
#[repr(C)]
pub struct sg_codel {
    _private: [u8; 0],
}
/// Router queue + `relay_inet_in` per host (relay/mod.rs:72-288).
#[repr(C)]
pub struct sg_inbound {
    _private: [u8; 0],
}
/// Interface FIFO + `relay_inet_out` per host (relay/mod.rs:111-275).
#[repr(C)]
pub struct sg_outbound {
    _private: [u8; 0],
}

// ---------------------------------------------------------------------------
// Structs
// ---------------------------------------------------------------------------
/// Edge list in GML edge order; node indices are petgraph `NodeIndex` values.
#[repr(C)]
#[derive(Debug, Clone, Copy)]
pub struct sg_graph {
    pub n_nodes: u32,
    pub n_edges: u32,
    pub edge_src: *const u32,
    pub edge_dst: *const u32,
    pub edge_latency_ns: *const u64,
    pub edge_packet_loss: *const f32,
    /// optional (null): GML ids, for messages
    pub node_gml_id: *const u32,
    pub directed: u8,
}

/// Zero-copy view of an `sg_routing_info`: cells `(latency_ns << 32) | bits(loss)`.
#[repr(C)]
#[derive(Debug, Clone, Copy)]
pub struct sg_routing_view {
    pub n: u32,
    pub node_ids: *const u32,
    pub cells: *const u64,
    pub n_wide: u64,
    pub pinned: u32,
}

/// A routing-table shard resident on the device (rows `[row_begin, row_begin + n_rows)`).
#[repr(C)]
#[derive(Debug, Clone, Copy)]
pub struct sg_table {
    pub latency_ns: *const u64,
    pub packet_loss: *const f32,
    pub n_cols: u32,
    pub row_begin: u32,
    pub n_rows: u32,
    /// null = the two-array form
    pub path_key: *const u64,
}

/// Round clock (EmulatedTime ns): the worker's barrier (worker.rs:262-268), sim end, bootstrap end.
#[repr(C)]
#[derive(Debug, Clone, Copy, Default)]
pub struct sg_round {
    pub round_end_ns: u64,
    pub sim_end_ns: u64,
    pub bootstrap_end_ns: u64,
}

/// One round's sent packets (device SoA, grouped by ascending source host, send order).
#[repr(C)]
#[derive(Debug, Clone, Copy)]
pub struct sg_packets {
    pub n_packets: u32,
    pub src_host: *const u32,
    pub dst_ipv4: *const u32,
    pub payload_len: *const u32,
    pub send_time_ns: *const u64,
    /// null = none: other consumers' steps of the host's RNG stream (host.rs:645-647)
    pub rng_skip: *const u32,
}

/// Device outputs of `sg_deliver_round`.
#[repr(C)]
#[derive(Debug, Clone, Copy)]
pub struct sg_deliveries {
    pub status: *mut u8,
    pub deliver_time_ns: *mut u64,
    pub event_id: *mut u64,
    pub dst_order: *mut u32,
    pub dst_offsets: *mut u32,
}

/// The round minima `Manager::run` folds (worker.rs:372,388).
#[repr(C)]
#[derive(Debug, Clone, Copy, Default)]
pub struct sg_round_stats {
    pub n_delivered: u64,
    pub min_deliver_time_ns: u64,
    pub min_used_latency_ns: u64,
}

/// One delivered packet on its way to the destination's owner rank (32 bytes).
#[repr(C)]
#[derive(Debug, Clone, Copy, Default)]
pub struct sg_record {
    pub deliver_time_ns: u64,
    /// (src_host << 32) | k, k = rank among src_host's delivered packets this round
    pub order_key: u64,
    pub event_id: u64,
    pub packet: u32,
    pub dst_host: u32,
}

/// A batch of CoDel push / pop events (device arrays, grouped by ascending host).
#[repr(C)]
#[derive(Debug, Clone, Copy)]
pub struct sg_codel_events {
    pub n_events: u32,
    pub host: *const u32,
    /// `SG_CODEL_PUSH` | `SG_CODEL_POP`
    pub kind: *const u8,
    pub time_ns: *const u64,
    pub packet: *const u32,
    pub len: *const u32,
}

/// Per-host CoDel state (host arrays) for checkpoints and tests.
#[repr(C)]
#[derive(Debug, Clone, Copy)]
pub struct sg_codel_state {
    pub flags: *mut u8,
    pub interval_end: *mut u64,
    pub drop_next: *mut u64,
    pub cur_drops: *mut u64,
    pub prev_drops: *mut u64,
    pub bytes: *mut u64,
    pub head: *mut u32,
    pub tail: *mut u32,
    pub ring_packet: *mut u32,
    pub ring_time: *mut u64,
    pub ring_len: *mut u32,
}

/// A window's Packet events (device arrays, grouped by ascending host, EventQueue order).
#[repr(C)]
#[derive(Debug, Clone, Copy)]
pub struct sg_inbound_arrivals {
    pub n: u32,
    pub host: *const u32,
    pub time_ns: *const u64,
    pub packet: *const u32,
    pub len: *const u32,
}

/// Per-host relay and token-bucket state (host arrays).
#[repr(C)]
#[derive(Debug, Clone, Copy)]
pub struct sg_inbound_relay_state {
    pub flags: *mut u8,
    pub task_time: *mut u64,
    pub cached_packet: *mut u32,
    pub cached_len: *mut u32,
    pub tb_capacity: *mut u64,
    pub tb_balance: *mut u64,
    pub tb_increment: *mut u64,
    pub tb_last_refill: *mut u64,
    /// ABI 6, may be null: the pending forward task's event id (host.rs:649-653)
    pub task_event_id: *mut u64,
    /// ABI 6, may be null: the time that task was scheduled at
    pub task_created_ns: *mut u64,
}

/// A window's sends (device arrays, grouped by ascending host, interface order).
#[repr(C)]
#[derive(Debug, Clone, Copy)]
pub struct sg_outbound_sends {
    pub n: u32,
    pub host: *const u32,
    pub time_ns: *const u64,
    pub packet: *const u32,
    pub len: *const u32,
    pub payload_len: *const u32,
    pub dst_ipv4: *const u32,
    /// ABI 6, optional (null, or both): the sending event's id (u64::MAX: a Packet event)
    pub event_id: *const u64,
    pub event_created_ns: *const u64,
}

/// The packets an outbound window handed to `send_packet` (a delivery round's `sg_packets`).
#[repr(C)]
#[derive(Debug, Clone, Copy)]
pub struct sg_outbound_sent {
    pub cap: u32,
    pub src_host: *mut u32,
    pub dst_ipv4: *mut u32,
    pub payload_len: *mut u32,
    pub send_time_ns: *mut u64,
    pub packet: *mut u32,
}

/// Per-host interface FIFO (host arrays); a cached packet is the slot at head - 1.
#[repr(C)]
#[derive(Debug, Clone, Copy)]
pub struct sg_outbound_queue_state {
    pub head: *mut u32,
    pub tail: *mut u32,
    pub ring_packet: *mut u32,
    pub ring_len: *mut u32,
    pub ring_payload_len: *mut u32,
    pub ring_dst: *mut u32,
}

// ---------------------------------------------------------------------------
// Constants
// ---------------------------------------------------------------------------
/// Checked against `sg_abi_version()` at startup.
pub const SG_ABI_VERSION: i32 = 7;

// sg_status
pub const SG_OK: i32 = 0;
/// graph/mod.rs:266-268 "No edge connecting node {} to {}"
pub const SG_ERR_NO_EDGE: i32 = 1;
/// graph/mod.rs:269-275 "More than one edge connecting node {} to {}"
pub const SG_ERR_MULTI_EDGE: i32 = 2;
/// graph/mod.rs:219 (a panic in the reference)
pub const SG_ERR_UNREACHABLE: i32 = 3;
pub const SG_ERR_OOM: i32 = 4;
pub const SG_ERR_INVALID_ARG: i32 = 5;
pub const SG_ERR_DEVICE: i32 = 6;
/// NetworkGraph::parse / ShadowEdge::try_from (graph/mod.rs:72-181)
pub const SG_ERR_PARSE: i32 = 7;
pub const SG_ERR_UNSORTED: i32 = 8;
/// IpAssignment::assign_ip (graph/mod.rs:383-394)
pub const SG_ERR_DUPLICATE_IP: i32 = 9;
pub const SG_ERR_CAPACITY: i32 = 10;
/// EmulatedTime + SimulationTime past EMUTIME_MAX (a panic in the reference, emulated_time.rs:121-126)
pub const SG_ERR_TIME_OVERFLOW: i32 = 11;
/// sg_comm_*: RCCL could not be opened
pub const SG_ERR_UNSUPPORTED: i32 = 12;

pub const SG_TIMERS_ON: u32 = 1;
pub const SG_TIMERS_COUNT_WORK: u32 = 2;
/// network.use_shortest_path (configuration.rs:315-326)
pub const SG_ROUTE_SHORTEST_PATH: u32 = 1;
pub const SG_ROUTE_OUT_DEVICE: u32 = 2;
pub const SG_CELL_WIDE: u32 = 0xFFFF_FFFF;
pub const SG_COMM_ID_BYTES: usize = 128;

// sg_deliveries.status
pub const SG_PKT_DELIVERED: u8 = 0;
pub const SG_PKT_DROP_LOSS: u8 = 1;
pub const SG_PKT_DROP_NO_DST: u8 = 2;
pub const SG_PKT_SIM_END: u8 = 3;
// sg_codel_events.kind
pub const SG_CODEL_PUSH: u8 = 0;
pub const SG_CODEL_POP: u8 = 1;
// router / relay packet fates
pub const SG_CODEL_QUEUED: u8 = 0;
pub const SG_CODEL_DEQUEUED: u8 = 1;
/// PacketStatus::RouterDropped
pub const SG_CODEL_DROPPED: u8 = 2;
pub const SG_OUT_QUEUED: u8 = 0;
/// to the router: Worker::send_packet
pub const SG_OUT_SENT: u8 = 1;
/// dst == own address: back to the interface
pub const SG_OUT_LOCAL: u8 = 2;

// ---------------------------------------------------------------------------
// Entry points (in the header's order)
// ---------------------------------------------------------------------------
unsafe extern "C" {
    pub fn sg_abi_version() -> i32;

    // ---- context -------------------------------------------------------------
    pub fn sg_ctx_create(device: i32, out: *mut *mut sg_ctx) -> i32;
    pub fn sg_ctx_destroy(ctx: *mut sg_ctx);
    /// An existing hipStream_t (e.g. the caller's), or null for the context's own stream.
    pub fn sg_ctx_set_stream(ctx: *mut sg_ctx, hip_stream: *mut c_void) -> i32;
    pub fn sg_ctx_stream(ctx: *const sg_ctx) -> *mut c_void;
    pub fn sg_ctx_synchronize(ctx: *mut sg_ctx) -> i32;
    pub fn sg_ctx_last_error(ctx: *const sg_ctx) -> *const c_char;
    pub fn sg_ctx_last_error_pair(ctx: *const sg_ctx, row: *mut u32, col: *mut u32);
    pub fn sg_ctx_enable_timers(ctx: *mut sg_ctx, enable: i32) -> i32;
    pub fn sg_ctx_read_timer(ctx: *mut sg_ctx, kernel: *const c_char, total_ms: *mut f64, launches: *mut u64,
                             work: *mut f64) -> i32;

    // ---- GML ingest: load_network_graph + NetworkGraph::parse (graph/mod.rs:134-181, 483-513) ----
    pub fn sg_gml_parse(text: *const c_char, len: usize, out: *mut *mut sg_gml, err: *mut c_char, err_len: usize)
        -> i32;
    pub fn sg_gml_parse_threads(text: *const c_char, len: usize, threads: u32, out: *mut *mut sg_gml,
                                err: *mut c_char, err_len: usize) -> i32;
    pub fn sg_gml_load(path: *const c_char, compression: u32, threads: u32, out: *mut *mut sg_gml, err: *mut c_char,
                       err_len: usize) -> i32;
    /// The parsed edge list, borrowed until sg_gml_destroy.
    pub fn sg_gml_graph(g: *const sg_gml, out: *mut sg_graph) -> i32;
    /// NetworkGraph::node_id_to_index (graph/mod.rs:126-128).
    pub fn sg_gml_node_index(g: *const sg_gml, gml_id: u32, out_index: *mut u32) -> i32;
    pub fn sg_gml_destroy(g: *mut sg_gml);

    // ---- routing-table build: compute_shortest_paths / get_direct_paths (graph/mod.rs:183-252) ----
    pub fn sg_net_create(ctx: *mut sg_ctx, g: *const sg_graph, out: *mut *mut sg_net) -> i32;
    pub fn sg_net_destroy(net: *mut sg_net);
    pub fn sg_routing_build(ctx: *mut sg_ctx, net: *mut sg_net, nodes: *const u32, n_used: u32, row_begin: u32,
                            row_end: u32, flags: u32, out_latency_ns: *mut u64, out_packet_loss: *mut f32) -> i32;
    /// RoutingInfo::get_smallest_latency_ns (graph/mod.rs:478-480) over device latencies.
    pub fn sg_routing_min_latency(ctx: *mut sg_ctx, d_latency_ns: *const u64, count: usize, out_min: *mut u64)
        -> i32;

    // ---- host-side dense RoutingInfo: generate_routing_info (sim_config.rs:411-448) ----
    pub fn sg_routing_info_create(n_used: u32, node_ids: *const u32, out: *mut *mut sg_routing_info) -> i32;
    pub fn sg_routing_info_destroy(ri: *mut sg_routing_info);
    pub fn sg_routing_info_fill(ctx: *mut sg_ctx, net: *mut sg_net, nodes: *const u32, flags: u32,
                                ri: *mut sg_routing_info) -> i32;
    /// Rows all-gathered from other ranks' sg_routing_build (sg_comm_allgather_rows).
    pub fn sg_routing_info_set_rows(ri: *mut sg_routing_info, row_begin: u32, row_end: u32, latency_ns: *const u64,
                                    packet_loss: *const f32) -> i32;
    pub fn sg_routing_info_view(ri: *const sg_routing_info, out: *mut sg_routing_view) -> i32;
    pub fn sg_routing_info_rows(ri: *const sg_routing_info, row_begin: u32, row_end: u32, latency_ns: *mut u64,
                                packet_loss: *mut f32) -> i32;
    pub fn sg_routing_info_index(ri: *const sg_routing_info, node_id: u32, row: *mut u32) -> i32;
    /// RoutingInfo::path (graph/mod.rs:448-450): 1 = Some, 0 = None.
    pub fn sg_routing_info_path(ri: *const sg_routing_info, start: u32, end: u32, latency_ns: *mut u64,
                                packet_loss: *mut f32) -> i32;
    pub fn sg_routing_info_smallest_latency(ri: *const sg_routing_info, out: *mut u64) -> i32;
    /// RoutingInfo::increment_packet_count (graph/mod.rs:453-460).
    pub fn sg_routing_info_increment_packet_count(ri: *mut sg_routing_info, start: u32, end: u32) -> i32;
    pub fn sg_routing_info_packet_count(ri: *const sg_routing_info, start: u32, end: u32) -> u64;
    /// IpAssignment (graph/mod.rs:354-430).
    pub fn sg_routing_info_set_addresses(ri: *mut sg_routing_info, n_addrs: u32, ipv4: *const u32,
                                         node_id: *const u32) -> i32;
    /// worker_getLatency / worker_isRoutable (worker.rs:651-684): network-order addresses.
    pub fn sg_worker_get_latency(ri: *const sg_routing_info, src_be: u32, dst_be: u32, latency_ns: *mut u64) -> i32;
    pub fn sg_worker_get_reliability(ri: *const sg_routing_info, src_be: u32, dst_be: u32, reliability: *mut f32)
        -> i32;
    pub fn sg_worker_is_routable(ri: *const sg_routing_info, src_be: u32, dst_be: u32) -> i32;

    // ---- packet delivery: Worker::send_packet + push_packet_to_host (worker.rs:322-397, 597-607) ----
    pub fn sg_hosts_create(ctx: *mut sg_ctx, n_hosts: u32, host_ipv4: *const u32, host_route_idx: *const u32,
                           host_seed: *const u64, out: *mut *mut sg_hosts) -> i32;
    pub fn sg_hosts_get_state(hosts: *mut sg_hosts, rng_state: *mut u64, event_ctr: *mut u64) -> i32;
    pub fn sg_hosts_set_state(hosts: *mut sg_hosts, rng_state: *const u64, event_ctr: *const u64) -> i32;
    pub fn sg_hosts_skip(hosts: *mut sg_hosts, n: u32, host_ids: *const u32, steps: *const u64) -> i32;
    pub fn sg_hosts_destroy(hosts: *mut sg_hosts);
    /// RoutingInfo::increment_packet_count on the device (ABI 7); null turns counting off.
    pub fn sg_ctx_set_packet_counters(ctx: *mut sg_ctx, counts: *mut u64, n_cells: u64) -> i32;
    pub fn sg_table_pack(ctx: *mut sg_ctx, table: *const sg_table, out_key: *mut u64, out_packable: *mut u32) -> i32;
    pub fn sg_deliver_round(ctx: *mut sg_ctx, hosts: *mut sg_hosts, table: *const sg_table, round: *const sg_round,
                            packets: *const sg_packets, out: *mut sg_deliveries, stats: *mut sg_round_stats) -> i32;

    // ---- sharded delivery: source half, exchange, destination half ----
    pub fn sg_deliver_source(ctx: *mut sg_ctx, hosts: *mut sg_hosts, table: *const sg_table, round: *const sg_round,
                             packets: *const sg_packets, status: *mut u8, deliver_time_ns: *mut u64,
                             event_id: *mut u64, host_owner: *const u32, n_ranks: u32, send: *mut sg_record,
                             send_counts: *mut u32, stats: *mut sg_round_stats) -> i32;
    pub fn sg_deliver_bucket(ctx: *mut sg_ctx, recv: *const sg_record, n_records: u32, host_local: *const u32,
                             n_hosts: u32, n_local_hosts: u32, dst_order: *mut u32, dst_offsets: *mut u32) -> i32;
    // the fixed-split exchange (one host synchronisation per round)
    pub fn sg_deliver_source_padded(ctx: *mut sg_ctx, hosts: *mut sg_hosts, table: *const sg_table,
                                    round: *const sg_round, packets: *const sg_packets, status: *mut u8,
                                    deliver_time_ns: *mut u64, event_id: *mut u64, host_owner: *const u32,
                                    n_ranks: u32, cap: u32, send_padded: *mut sg_record, send: *mut sg_record,
                                    xrow: *mut u64) -> i32;
    pub fn sg_deliver_bucket_padded(ctx: *mut sg_ctx, recv_padded: *const sg_record, n_ranks: u32, cap: u32,
                                    xall: *const u64, rank: u32, host_local: *const u32, n_hosts: u32,
                                    n_local_hosts: u32, dst_order: *mut u32, dst_offsets: *mut u32,
                                    stats: *mut sg_round_stats, recv_counts: *mut u32, pair_max: *mut u32) -> i32;
    pub fn sg_deliver_pad_to_compact(ctx: *mut sg_ctx, send_padded: *const sg_record, n_ranks: u32, cap: u32,
                                     xrow: *const u64, send: *mut sg_record) -> i32;

    // ---- collectives of the sharded path over RCCL (ABI 7, on the context's stream) ----
    pub fn sg_comm_unique_id(id: *mut u8) -> i32;
    pub fn sg_comm_create(ctx: *mut sg_ctx, id: *const u8, n_ranks: u32, rank: u32, out: *mut *mut sg_comm) -> i32;
    pub fn sg_comm_destroy(comm: *mut sg_comm);
    pub fn sg_comm_allgather_rows(comm: *mut sg_comm, lat: *mut u64, loss: *mut f32, rows_per_rank: u32,
                                  n_used: u32) -> i32;
    pub fn sg_comm_exchange_padded(comm: *mut sg_comm, send_padded: *const sg_record, recv_padded: *mut sg_record,
                                   cap: u32, xrow: *const u64, xall: *mut u64) -> i32;
    pub fn sg_comm_alltoallv_records(comm: *mut sg_comm, send: *const sg_record, send_counts: *const u32,
                                     recv: *mut sg_record, recv_counts: *const u32) -> i32;
    pub fn sg_comm_allgather_u64(comm: *mut sg_comm, mine: *const u64, all: *mut u64, n: u32) -> i32;

    // ---- router inbound CoDel queues (router/mod.rs:15-58, codel_queue.rs) ----
    pub fn sg_codel_create(ctx: *mut sg_ctx, n_hosts: u32, ring_cap: u32, out: *mut *mut sg_codel) -> i32;
    pub fn sg_codel_destroy(q: *mut sg_codel);
    pub fn sg_codel_run(ctx: *mut sg_ctx, q: *mut sg_codel, ev: *const sg_codel_events, pop_result: *mut u32,
                        pkt_status: *mut u8, n_packets: u32, n_dropped: *mut u64) -> i32;
    pub fn sg_codel_ring_cap(q: *const sg_codel) -> u32;
    pub fn sg_codel_get_state(q: *mut sg_codel, out: *mut sg_codel_state) -> i32;
    pub fn sg_codel_set_state(q: *mut sg_codel, input: *const sg_codel_state) -> i32;

    // ---- inbound pipeline: router queue -> relay_inet_in (host.rs:781-786, relay/mod.rs:72-288) ----
    pub fn sg_inbound_create(ctx: *mut sg_ctx, n_hosts: u32, bw_down_bits: *const u64, ring_cap: u32,
                             out: *mut *mut sg_inbound) -> i32;
    pub fn sg_inbound_destroy(ib: *mut sg_inbound);
    pub fn sg_inbound_ring_cap(ib: *const sg_inbound) -> u32;
    pub fn sg_inbound_run(ctx: *mut sg_ctx, ib: *mut sg_inbound, arr: *const sg_inbound_arrivals, window_end_ns: u64,
                          bootstrap_end_ns: u64, sim_end_ns: u64, event_ctr: *mut u64, fwd_time: *mut u64,
                          pkt_status: *mut u8, n_packets: u32, n_dropped: *mut u64) -> i32;
    /// ABI 7: this call's arrivals' fates in arrival order.
    pub fn sg_inbound_run_ordered(ctx: *mut sg_ctx, ib: *mut sg_inbound, arr: *const sg_inbound_arrivals,
                                  window_end_ns: u64, bootstrap_end_ns: u64, sim_end_ns: u64, event_ctr: *mut u64,
                                  fwd_time: *mut u64, pkt_status: *mut u8, n_packets: u32, arr_fwd_time: *mut u64,
                                  arr_status: *mut u8, n_dropped: *mut u64) -> i32;
    pub fn sg_inbound_get_state(ib: *mut sg_inbound, queue: *mut sg_codel_state, relay: *mut sg_inbound_relay_state)
        -> i32;

    // ---- outbound pipeline: interface -> relay_inet_out -> router (relay/mod.rs:111-275) ----
    pub fn sg_outbound_create(ctx: *mut sg_ctx, n_hosts: u32, host_ipv4: *const u32, bw_up_bits: *const u64,
                              ring_cap: u32, out: *mut *mut sg_outbound) -> i32;
    pub fn sg_outbound_destroy(ob: *mut sg_outbound);
    pub fn sg_outbound_ring_cap(ob: *const sg_outbound) -> u32;
    pub fn sg_outbound_run(ctx: *mut sg_ctx, ob: *mut sg_outbound, sends: *const sg_outbound_sends,
                           window_end_ns: u64, bootstrap_end_ns: u64, sim_end_ns: u64, event_ctr: *mut u64,
                           fwd_time: *mut u64, pkt_status: *mut u8, n_packets: u32, sent: *mut sg_outbound_sent,
                           n_sent: *mut u32) -> i32;
    pub fn sg_outbound_get_state(ob: *mut sg_outbound, queue: *mut sg_outbound_queue_state,
                                 relay: *mut sg_inbound_relay_state) -> i32;

    /// The device array of the hosts' event-id counters (Host::event_id_counter).
    pub fn sg_hosts_event_ctr(hosts: *mut sg_hosts) -> *mut u64;
}
