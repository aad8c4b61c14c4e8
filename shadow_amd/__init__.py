"""shadow_amd -- MI355X-native network core for the Shadow simulator.

Two stages of Shadow's network core run as HIP kernels for gfx950 behind the
C ABI in include/shadow_gpu.h (libshadow_gpu.so):

* routing-table build (NetworkGraph::compute_shortest_paths / get_direct_paths,
  src/main/network/graph/mod.rs:183-252) -> `graph.NetworkGraph`;
* per-round packet delivery (Worker::send_packet, src/main/core/worker.rs:322-397)
  -> `worker.deliver_round`.

There is no CPU fallback: if libshadow_gpu.so is missing, `load()` raises.
"""
from ._capi import LIB_PATH, ShadowGpuError, ShadowGpuUnavailable, load  # noqa: F401
from .graph import (Context, IpAssignment, NetworkGraph, PathProperties, PathTable,  # noqa: F401
                    RoutingInfo, default_context, generate_routing_info, ipv4_to_u32, u32_to_ipv4)

__all__ = ["Context", "NetworkGraph", "PathProperties", "PathTable", "RoutingInfo", "IpAssignment",
           "generate_routing_info", "default_context", "load", "ShadowGpuError", "ShadowGpuUnavailable",
           "ipv4_to_u32", "u32_to_ipv4", "LIB_PATH"]
