// sg_comm.hip -- the collectives of the sharded path, behind the C ABI, over RCCL (xGMI).
//
// One communicator per rank (one process per GPU), bound to an sg_ctx: its device and
// its stream, so every exchange is ordered with the library's kernels and needs no host
// synchronisation.  The reference hands packets between worker threads
// (Worker::push_packet_to_host, worker.rs:597-607; the manager's round loop,
// manager.rs:415-501) and builds the routing table once per simulation
// (sim_config.rs:137-141, graph/mod.rs:183-228); sharded over GPUs these become
//   * sg_comm_allgather_rows: the row blocks of the table (one all-gather in place),
//   * sg_comm_exchange_padded: the fixed-split round exchange (the [stats, counts]
//     rows all-gathered, the record blocks all-to-all),
//   * sg_comm_alltoallv_records: the exact exchange (host-known counts),
//   * sg_comm_allgather_u64: small rows (round scalars, counts).
// RCCL is opened at run time (dlopen of librccl.so.1: in a process that already holds
// one, e.g. torch's, that copy; else the system library), so the library loads and
// every other entry point works without it.  A caller without torch (the Rust side of
// INTEGRATION.md) gets the unique id from sg_comm_unique_id on one rank and passes the
// 128 bytes to the others over its own channel.
#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <string>

#include <rccl/rccl.h>

#include "sg_internal.h"

namespace {

struct Rccl {
  bool ok = false;
  std::string why;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      r.why = std::string("librccl.so.1 not found: ") + dlerror();
      return;
    }
    auto sym = [&](const char* name) {
      void* p = dlsym(h, name);
      if (!p && r.why.empty()) r.why = std::string("librccl.so.1 lacks ") + name;
      return p;
    };
    r.get_unique_id = (decltype(r.get_unique_id))sym("ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))sym("ncclCommInitRank");
    r.comm_destroy = (decltype(r.comm_destroy))sym("ncclCommDestroy");
    r.all_gather = (decltype(r.all_gather))sym("ncclAllGather");
    r.send = (decltype(r.send))sym("ncclSend");
    r.recv = (decltype(r.recv))sym("ncclRecv");
    r.group_start = (decltype(r.group_start))sym("ncclGroupStart");
    r.group_end = (decltype(r.group_end))sym("ncclGroupEnd");
    r.error_string = (decltype(r.error_string))sym("ncclGetErrorString");
    r.ok = r.why.empty();
  });
  return r;
}

void need_rccl() {
  const Rccl& r = rccl();
  if (!r.ok) throw sg::Error(SG_ERR_UNSUPPORTED, "RCCL unavailable: " + r.why);
}

void nccl_check(ncclResult_t e, const char* what) {
  if (e != ncclSuccess)
    throw sg::Error(SG_ERR_DEVICE, std::string(what) + ": " + (rccl().error_string ? rccl().error_string(e) : "?"));
}

}  // namespace

struct sg_comm {
  sg_ctx* ctx = nullptr;
  ncclComm_t comm = nullptr;
  uint32_t n_ranks = 0, rank = 0;
};

extern "C" {

int32_t sg_comm_unique_id(uint8_t* id) {
  if (!id) return SG_ERR_INVALID_ARG;
  try {
    need_rccl();
    ncclUniqueId u;
    nccl_check(rccl().get_unique_id(&u), "ncclGetUniqueId");
    memcpy(id, u.internal, SG_COMM_ID_BYTES);
    return SG_OK;
  } catch (const sg::Error& e) {
    return e.code;
  }
}

int32_t sg_comm_create(sg_ctx* ctx, const uint8_t* id, uint32_t n_ranks, uint32_t rank, sg_comm** out) {
  if (!ctx || !id || !out || !n_ranks || rank >= n_ranks) return SG_ERR_INVALID_ARG;
  *out = nullptr;
  return sg::guarded(ctx, [&] {
    need_rccl();
    ncclUniqueId u;
    memcpy(u.internal, id, SG_COMM_ID_BYTES);
    auto* c = new sg_comm();
    c->ctx = ctx;
    c->n_ranks = n_ranks;
    c->rank = rank;
    const ncclResult_t e = rccl().comm_init_rank(&c->comm, (int)n_ranks, u, (int)rank);
    if (e != ncclSuccess) {
      delete c;
      nccl_check(e, "ncclCommInitRank");
    }
    *out = c;
  });
}

void sg_comm_destroy(sg_comm* c) {
  if (!c) return;
  if (c->comm && rccl().ok) {
    (void)hipStreamSynchronize(c->ctx->stream);
    (void)rccl().comm_destroy(c->comm);
  }
  delete c;
}

int32_t sg_comm_allgather_rows(sg_comm* c, uint64_t* lat, float* loss, uint32_t rows_per_rank, uint32_t n_used) {
  if (!c || (!lat && !loss)) return SG_ERR_INVALID_ARG;
  return sg::guarded(c->ctx, [&] {
    const size_t per = (size_t)rows_per_rank * n_used;
    if (!per) return;
    // in place: rank r's block is its own send buffer (ncclAllGather's in-place form)
    if (lat)
      nccl_check(rccl().all_gather(lat + per * c->rank, lat, per, ncclUint64, c->comm, c->ctx->stream),
                 "ncclAllGather (latency rows)");
    if (loss)
      nccl_check(rccl().all_gather(loss + per * c->rank, loss, per, ncclFloat32, c->comm, c->ctx->stream),
                 "ncclAllGather (loss rows)");
  });
}

int32_t sg_comm_allgather_u64(sg_comm* c, const uint64_t* mine, uint64_t* all, uint32_t n) {
  if (!c || !mine || !all) return SG_ERR_INVALID_ARG;
  return sg::guarded(c->ctx, [&] {
    if (n) nccl_check(rccl().all_gather(mine, all, n, ncclUint64, c->comm, c->ctx->stream), "ncclAllGather");
  });
}

int32_t sg_comm_exchange_padded(sg_comm* c, const sg_record* send_padded, sg_record* recv_padded, uint32_t cap,
                                const uint64_t* xrow, uint64_t* xall) {
  if (!c || !xrow || !xall || (cap && (!send_padded || !recv_padded))) return SG_ERR_INVALID_ARG;
  return sg::guarded(c->ctx, [&] {
    const Rccl& r = rccl();
    hipStream_t st = c->ctx->stream;
    nccl_check(r.all_gather(xrow, xall, 3 + c->n_ranks, ncclUint64, c->comm, st), "ncclAllGather (round rows)");
    if (!cap) return;
    // equal blocks of cap records per rank pair: grouped point-to-point sends and receives
    // (an all-to-all over xGMI's point-to-point links)
    const size_t words = (size_t)cap * (sizeof(sg_record) / 8);
    nccl_check(r.group_start(), "ncclGroupStart");
    for (uint32_t p = 0; p < c->n_ranks; p++) {
      nccl_check(r.send((const uint64_t*)(send_padded + (size_t)p * cap), words, ncclUint64, (int)p, c->comm, st),
                 "ncclSend");
      nccl_check(r.recv((uint64_t*)(recv_padded + (size_t)p * cap), words, ncclUint64, (int)p, c->comm, st),
                 "ncclRecv");
    }
    nccl_check(r.group_end(), "ncclGroupEnd");
  });
}

int32_t sg_comm_alltoallv_records(sg_comm* c, const sg_record* send, const uint32_t* send_counts, sg_record* recv,
                                  const uint32_t* recv_counts) {
  if (!c || !send_counts || !recv_counts) return SG_ERR_INVALID_ARG;
  return sg::guarded(c->ctx, [&] {
    const Rccl& r = rccl();
    hipStream_t st = c->ctx->stream;
    size_t so = 0, ro = 0;
    for (uint32_t p = 0; p < c->n_ranks; p++) {
      so += send_counts[p];
      ro += recv_counts[p];
    }
    if ((so && !send) || (ro && !recv)) throw sg::Error(SG_ERR_INVALID_ARG, "null record buffer");
    constexpr size_t W = sizeof(sg_record) / 8;
    so = ro = 0;
    nccl_check(r.group_start(), "ncclGroupStart");
    for (uint32_t p = 0; p < c->n_ranks; p++) {
      if (send_counts[p])
        nccl_check(r.send((const uint64_t*)(send + so), (size_t)send_counts[p] * W, ncclUint64, (int)p, c->comm, st),
                   "ncclSend");
      if (recv_counts[p])
        nccl_check(r.recv((uint64_t*)(recv + ro), (size_t)recv_counts[p] * W, ncclUint64, (int)p, c->comm, st),
                   "ncclRecv");
      so += send_counts[p];
      ro += recv_counts[p];
    }
    nccl_check(r.group_end(), "ncclGroupEnd");
  });
}

}  // extern "C"
