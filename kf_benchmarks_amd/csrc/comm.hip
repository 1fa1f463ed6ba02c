// Native RCCL communicator: the collectives of data-parallel training over
// xGMI, owned by this library instead of torch's ProcessGroupNCCL.
//
// Replaces the reference's NCCL / CollectiveOps / Horovod / KungFu device
// collectives (tcb/allreduce.py:297-299 NcclAllReduce, tcb/variable_mgr.py:
// 566-612 broadcast, tcb/benchmark_cnn.py:3122-3130 hvd.allreduce): one
// communicator per process (one process per GPU), created with
// ncclCommInitRank from a unique id the Python side exchanges over the job's
// TCP store (parallel/rccl.py).  Every collective is an ordinary entry point
// taking raw device pointers and the stream to run on, so a recorded launch
// tape (csrc/tape.hip) replays a multi-GPU step's gradient all-reduces
// exactly like its kernels.
//
// RCCL is loaded at run time: the copy torch already mapped if there is one
// (one RCCL per process), else librccl.so.1 from the library path.
#include "common.h"

#include <dlfcn.h>

#include <cstring>
#include <mutex>

namespace kfb {
namespace rccl {

typedef int ncclResult_t;
typedef void* ncclComm_t;
struct UniqueId {
  char internal[128];
};

struct Api {
  bool ok = false;
  ncclResult_t (*get_unique_id)(UniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, UniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) =
      nullptr;
  ncclResult_t (*reduce)(const void*, void*, size_t, int, int, int, ncclComm_t, hipStream_t) =
      nullptr;
  ncclResult_t (*broadcast)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) =
      nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*reduce_scatter)(const void*, void*, size_t, int, int, ncclComm_t,
                                 hipStream_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

static Api& api() {
  static Api a;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
#define KFB_SYM(f, n) a.f = (decltype(a.f))dlsym(h, n)
    KFB_SYM(get_unique_id, "ncclGetUniqueId");
    KFB_SYM(comm_init_rank, "ncclCommInitRank");
    KFB_SYM(comm_destroy, "ncclCommDestroy");
    KFB_SYM(comm_abort, "ncclCommAbort");
    KFB_SYM(all_reduce, "ncclAllReduce");
    KFB_SYM(reduce, "ncclReduce");
    KFB_SYM(broadcast, "ncclBroadcast");
    KFB_SYM(all_gather, "ncclAllGather");
    KFB_SYM(reduce_scatter, "ncclReduceScatter");
    KFB_SYM(send, "ncclSend");
    KFB_SYM(recv, "ncclRecv");
    KFB_SYM(group_start, "ncclGroupStart");
    KFB_SYM(group_end, "ncclGroupEnd");
    KFB_SYM(async_error, "ncclCommGetAsyncError");
    KFB_SYM(error_string, "ncclGetErrorString");
#undef KFB_SYM
    a.ok = a.get_unique_id && a.comm_init_rank && a.comm_destroy && a.all_reduce && a.reduce &&
           a.broadcast && a.group_start && a.group_end;
  });
  return a;
}

// element type codes of the kernels (common.h) -> ncclDataType_t
static int nccl_dtype(int dt) {
  switch (dt) {
    case F32: return 7;   // ncclFloat32
    case BF16: return 9;  // ncclBfloat16
    case F16: return 6;   // ncclFloat16
    case 3: return 2;     // int32 (ncclInt32)
    case 4: return 8;     // float64 (ncclFloat64)
    default: return -1;
  }
}

// reduction codes: 0 sum, 1 prod, 2 max, 3 min (ncclRedOp_t)
static bool valid_op(int op) { return op >= 0 && op <= 3; }

// RCCL results are returned offset by 1000 so they cannot be mistaken for
// hipError_t codes by the caller (0 stays success).
static int rc(ncclResult_t r) {
  kfb::raw_taint();  // a recorded op that talks to RCCL replays through its entry point
  return r == 0 ? 0 : 1000 + r;
}

}  // namespace rccl
}  // namespace kfb

using namespace kfb::rccl;

KFB_API int kfb_rccl_available() { return api().ok ? 1 : 0; }

KFB_API const char* kfb_rccl_error_string(int code) {
  if (code >= 1000 && api().error_string) return api().error_string(code - 1000);
  return hipGetErrorString((hipError_t)code);
}

// 128-byte unique id of a new communicator (rank 0 creates it).
KFB_API int kfb_rccl_unique_id(char* out128) {
  if (!api().ok) return 999;
  UniqueId id;
  const int r = rc(api().get_unique_id(&id));
  if (r == 0) memcpy(out128, id.internal, sizeof(id.internal));
  return r;
}

// Creates this rank's communicator on ``device`` (collective over nranks).
KFB_API int kfb_rccl_init(int nranks, const char* id128, int rank, int device, void** comm) {
  if (!api().ok) return 999;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return e;
  UniqueId id;
  memcpy(id.internal, id128, sizeof(id.internal));
  ncclComm_t c = nullptr;
  const int r = rc(api().comm_init_rank(&c, nranks, id, rank));
  *comm = r == 0 ? c : nullptr;
  return r;
}

KFB_API int kfb_rccl_destroy(void* comm, int abort) {
  if (!api().ok || !comm) return 0;
  return rc(abort && api().comm_abort ? api().comm_abort(comm) : api().comm_destroy(comm));
}

KFB_API int kfb_rccl_async_error(void* comm) {
  if (!api().ok || !comm || !api().async_error) return 0;
  ncclResult_t e = 0;
  const int r = rc(api().async_error(comm, &e));
  return r ? r : rc(e);
}

// In place when send == recv.  count in elements.
KFB_API int kfb_rccl_all_reduce(void* comm, const void* send, void* recv, size_t count, int dtype,
                                int op, hipStream_t s) {
  const int dt = nccl_dtype(dtype);
  if (dt < 0 || !valid_op(op)) return hipErrorInvalidValue;
  return rc(api().all_reduce(send, recv, count, dt, op, comm, s));
}

KFB_API int kfb_rccl_reduce(void* comm, const void* send, void* recv, size_t count, int dtype,
                            int op, int root, hipStream_t s) {
  const int dt = nccl_dtype(dtype);
  if (dt < 0 || !valid_op(op)) return hipErrorInvalidValue;
  return rc(api().reduce(send, recv, count, dt, op, root, comm, s));
}

KFB_API int kfb_rccl_broadcast(void* comm, const void* send, void* recv, size_t count, int dtype,
                               int root, hipStream_t s) {
  const int dt = nccl_dtype(dtype);
  if (dt < 0) return hipErrorInvalidValue;
  return rc(api().broadcast(send, recv, count, dt, root, comm, s));
}

KFB_API int kfb_rccl_all_gather(void* comm, const void* send, void* recv, size_t count,
                                int dtype, hipStream_t s) {
  const int dt = nccl_dtype(dtype);
  if (dt < 0 || !api().all_gather) return hipErrorInvalidValue;
  return rc(api().all_gather(send, recv, count, dt, comm, s));
}

KFB_API int kfb_rccl_reduce_scatter(void* comm, const void* send, void* recv, size_t count,
                                    int dtype, int op, hipStream_t s) {
  const int dt = nccl_dtype(dtype);
  if (dt < 0 || !valid_op(op) || !api().reduce_scatter) return hipErrorInvalidValue;
  return rc(api().reduce_scatter(send, recv, count, dt, op, comm, s));
}

KFB_API int kfb_rccl_send(void* comm, const void* buf, size_t count, int dtype, int peer,
                          hipStream_t s) {
  const int dt = nccl_dtype(dtype);
  if (dt < 0 || !api().send) return hipErrorInvalidValue;
  return rc(api().send(buf, count, dt, peer, comm, s));
}

KFB_API int kfb_rccl_recv(void* comm, void* buf, size_t count, int dtype, int peer,
                          hipStream_t s) {
  const int dt = nccl_dtype(dtype);
  if (dt < 0 || !api().recv) return hipErrorInvalidValue;
  return rc(api().recv(buf, count, dt, peer, comm, s));
}

KFB_API int kfb_rccl_group_start() { return api().ok ? rc(api().group_start()) : 999; }
KFB_API int kfb_rccl_group_end() { return api().ok ? rc(api().group_end()) : 999; }
