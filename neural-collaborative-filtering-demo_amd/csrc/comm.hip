// RCCL collectives of the row-sharded step, issued straight from the C-ABI on the caller's HIP
// stream: the variable-split all-to-alls of the exchange phases (one grouped ncclSend/ncclRecv
// per peer) and the sum all-reduce of the flat dense gradient.
//
// Reference: the reference trains on one process; its scale-out is torchrec's sharded EBC
// (SURVEY §8(e)), whose input/output distribution is an all-to-all with per-rank splits.  These
// entry points carry the same exchanges as torch.distributed.all_to_all_single(out, in,
// recv_splits, send_splits) / all_reduce over RCCL, without the per-call work of the c10d layer
// (Work objects, stream-sync events, allocator stream bookkeeping): one ncclGroupStart/End per
// exchange on the stream the step's kernels run on.
//
// RCCL is not linked: its functions are resolved at first use from the librccl.so.1 already in
// the process (the one torch loads), so the communicators live in the same library instance as
// torch's own process groups.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include "ncf_common.h"

namespace {

struct Rccl {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
};

template <typename F>
bool bind(void* h, const char* name, F& fn) {
  fn = reinterpret_cast<F>(dlsym(h, name));
  return fn != nullptr;
}

Rccl load_rccl() {
  Rccl r;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) return r;
  r.ok = bind(h, "ncclGetUniqueId", r.get_unique_id) && bind(h, "ncclCommInitRank", r.comm_init_rank) &&
         bind(h, "ncclCommDestroy", r.comm_destroy) && bind(h, "ncclGroupStart", r.group_start) &&
         bind(h, "ncclGroupEnd", r.group_end) && bind(h, "ncclSend", r.send) &&
         bind(h, "ncclRecv", r.recv) && bind(h, "ncclAllReduce", r.all_reduce) &&
         bind(h, "ncclGetErrorString", r.error_string);
  return r;
}

const Rccl& rccl() {
  static const Rccl r = load_rccl();
  return r;
}

int rccl_fail(const char* what, ncclResult_t rc) {
  ncf_set_error("%s: RCCL error %d (%s)", what, (int)rc,
                rccl().error_string ? rccl().error_string(rc) : "?");
  return NCF_ERR_LAUNCH;
}

#define NCF_RCCL(what, expr)                        \
  do {                                              \
    const ncclResult_t rc_ = (expr);                \
    if (rc_ != ncclSuccess) return rccl_fail(what, rc_); \
  } while (0)

struct Comm {
  ncclComm_t comm;
  int world, rank;
};

}  // namespace

extern "C" int ncf_comm_available(void) { return rccl().ok ? 1 : 0; }

extern "C" int ncf_comm_unique_id(uint8_t* id, int64_t bytes) {
  NCF_CHECK_ARG(id && bytes >= NCCL_UNIQUE_ID_BYTES, "ncf_comm_unique_id: need %d bytes",
                NCCL_UNIQUE_ID_BYTES);
  NCF_CHECK_ARG(rccl().ok, "ncf_comm_unique_id: librccl not found in the process");
  ncclUniqueId u;
  NCF_RCCL("ncf_comm_unique_id", rccl().get_unique_id(&u));
  memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return NCF_OK;
}

extern "C" int ncf_comm_init(const uint8_t* id, int64_t bytes, int world, int rank, void** comm) {
  NCF_CHECK_ARG(id && bytes >= NCCL_UNIQUE_ID_BYTES && comm && world >= 1 && rank >= 0 &&
                    rank < world,
                "ncf_comm_init: bad args");
  NCF_CHECK_ARG(rccl().ok, "ncf_comm_init: librccl not found in the process");
  ncclUniqueId u;
  memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  NCF_RCCL("ncf_comm_init", rccl().comm_init_rank(&c, world, u, rank));
  *comm = new Comm{c, world, rank};
  return NCF_OK;
}

extern "C" int ncf_comm_destroy(void* comm) {
  if (!comm) return NCF_OK;
  Comm* c = static_cast<Comm*>(comm);
  const ncclResult_t rc = rccl().comm_destroy(c->comm);
  delete c;
  if (rc != ncclSuccess) return rccl_fail("ncf_comm_destroy", rc);
  return NCF_OK;
}

// recv[rows of peer p at recv offset] <- send[rows for p at send offset], offsets the prefix
// sums of the per-peer row counts (host arrays of `world` entries), rows of row_bytes bytes
extern "C" int ncf_comm_alltoallv(void* comm, const void* send, const int64_t* send_rows,
                                  void* recv, const int64_t* recv_rows, int64_t row_bytes,
                                  void* stream) {
  NCF_CHECK_ARG(comm && send_rows && recv_rows && row_bytes >= 1, "ncf_comm_alltoallv: bad args");
  const Comm* c = static_cast<const Comm*>(comm);
  hipStream_t st = (hipStream_t)stream;
  int64_t so = 0, ro = 0;
  for (int p = 0; p < c->world; ++p) {
    NCF_CHECK_ARG(send_rows[p] >= 0 && recv_rows[p] >= 0, "ncf_comm_alltoallv: negative count");
    so += send_rows[p];
    ro += recv_rows[p];
  }
  NCF_CHECK_ARG((so == 0 || send) && (ro == 0 || recv), "ncf_comm_alltoallv: null buffer");
  const char* sb = static_cast<const char*>(send);
  char* rb = static_cast<char*>(recv);
  // this rank's own share is a device copy on the stream (RCCL's send-to-self runs it through
  // its kernel at a fraction of the copy rate); RCCL carries only the peers' shares, and a
  // world of 1 launches no RCCL kernel at all
  int64_t so_self = 0, ro_self = 0;
  for (int p = 0; p < c->rank; ++p) {
    so_self += send_rows[p];
    ro_self += recv_rows[p];
  }
  NCF_CHECK_ARG(send_rows[c->rank] == recv_rows[c->rank], "ncf_comm_alltoallv: self counts differ");
  if (send_rows[c->rank] &&
      hipMemcpyAsync(rb + ro_self * row_bytes, sb + so_self * row_bytes,
                     (size_t)(send_rows[c->rank] * row_bytes), hipMemcpyDeviceToDevice, st) != hipSuccess) {
    ncf_set_error("ncf_comm_alltoallv: self copy failed");
    return NCF_ERR_LAUNCH;
  }
  if (c->world == 1) return NCF_OK;
  NCF_RCCL("ncf_comm_alltoallv(group start)", rccl().group_start());
  so = 0;
  ro = 0;
  for (int p = 0; p < c->world; ++p) {
    if (p == c->rank) {
      so += send_rows[p];
      ro += recv_rows[p];
      continue;
    }
    if (send_rows[p]) {
      const ncclResult_t rc =
          rccl().send(sb + so * row_bytes, (size_t)(send_rows[p] * row_bytes), ncclInt8, p, c->comm, st);
      if (rc != ncclSuccess) {
        rccl().group_end();
        return rccl_fail("ncf_comm_alltoallv(send)", rc);
      }
    }
    if (recv_rows[p]) {
      const ncclResult_t rc =
          rccl().recv(rb + ro * row_bytes, (size_t)(recv_rows[p] * row_bytes), ncclInt8, p, c->comm, st);
      if (rc != ncclSuccess) {
        rccl().group_end();
        return rccl_fail("ncf_comm_alltoallv(recv)", rc);
      }
    }
    so += send_rows[p];
    ro += recv_rows[p];
  }
  NCF_RCCL("ncf_comm_alltoallv(group end)", rccl().group_end());
  return NCF_OK;
}

extern "C" int ncf_comm_allreduce_sum_f32(void* comm, float* buf, int64_t n, void* stream) {
  NCF_CHECK_ARG(comm && n >= 0 && (n == 0 || buf), "ncf_comm_allreduce_sum_f32: bad args");
  if (n == 0) return NCF_OK;
  const Comm* c = static_cast<const Comm*>(comm);
  if (c->world == 1) return NCF_OK;   // the sum over one rank is the buffer itself
  NCF_RCCL("ncf_comm_allreduce_sum_f32",
           rccl().all_reduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, c->comm, (hipStream_t)stream));
  return NCF_OK;
}
