// Data-parallel gradient exchange: a native RCCL communicator over the
// ranks of one node and the ONE collective of the PPO update -- an in-place SUM all-reduce of the
// flat actor+critic gradient per optimizer step (the step all-reduced is ppo.py:120-135).
//
// The reference has no distributed code (no torch.distributed, no NCCL/MPI/Gloo).
//
// Why native and not torch.distributed: the collective is issued straight onto the caller's
// compute stream (ncclAllReduce(..., stream)), so a hipGraph capture of the optimizer loop records
// it like any kernel launch -- fused gradient -> all-reduce -> Adam tail replays as one graph with
// no host round trip per step.  The process group (torch.distributed, any backend) is only used
// once, to broadcast the 128-byte unique id from rank 0.
//
// RCCL is resolved at run time (dlopen), not linked: the library that torch.distributed already
// loaded into the process is reused when present (RTLD_NOLOAD on "librccl.so", the name torch's
// libtorch_hip.so records), otherwise ROCm's librccl.so.1; PPO_RCCL_LIB overrides the path.  So
// the engine loads on machines without RCCL and only ppo_comm_* fail there, with a message.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>

#include "common.h"
#include "ctx.h"

struct ppo_comm {
  ncclComm_t comm;
  int nranks, rank, device;
};

namespace ppo {
namespace {

struct RcclApi {
  void *lib = nullptr;
  const char *source = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*async_error)(ncclComm_t, ncclResult_t *) = nullptr;
  const char *(*error_string)(ncclResult_t) = nullptr;
  ncclResult_t (*get_version)(int *) = nullptr;
  ncclResult_t (*comm_count)(const ncclComm_t, int *) = nullptr;
  ncclResult_t (*comm_user_rank)(const ncclComm_t, int *) = nullptr;
  char err[256] = {0};
};

RcclApi g_rccl;
std::once_flag g_rccl_once;

void rccl_load() {
  RcclApi &r = g_rccl;
  const char *env = std::getenv("PPO_RCCL_LIB");
  if (env && *env) {
    r.lib = dlopen(env, RTLD_NOW | RTLD_LOCAL);
    r.source = "PPO_RCCL_LIB";
  }
  if (!r.lib) {  // the instance torch.distributed already loaded (libtorch_hip.so NEEDED entry)
    r.lib = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    r.source = "process (torch)";
  }
  if (!r.lib) {
    r.lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    r.source = "librccl.so.1";
  }
  if (!r.lib) {
    snprintf(r.err, sizeof(r.err), "RCCL not found: %s", dlerror());
    return;
  }
#define PPO_SYM(field, name)                                                         \
  r.field = reinterpret_cast<decltype(r.field)>(dlsym(r.lib, name));                 \
  if (!r.field) {                                                                    \
    snprintf(r.err, sizeof(r.err), "RCCL (%s) lacks %s", r.source, name);            \
    r.lib = nullptr;                                                                 \
    return;                                                                          \
  }
  PPO_SYM(get_unique_id, "ncclGetUniqueId")
  PPO_SYM(comm_init_rank, "ncclCommInitRank")
  PPO_SYM(comm_destroy, "ncclCommDestroy")
  PPO_SYM(all_reduce, "ncclAllReduce")
  PPO_SYM(async_error, "ncclCommGetAsyncError")
  PPO_SYM(error_string, "ncclGetErrorString")
  PPO_SYM(get_version, "ncclGetVersion")
  PPO_SYM(comm_count, "ncclCommCount")
  PPO_SYM(comm_user_rank, "ncclCommUserRank")
#undef PPO_SYM
}

const RcclApi *rccl() {
  std::call_once(g_rccl_once, rccl_load);
  return g_rccl.lib ? &g_rccl : nullptr;
}

}  // namespace
}  // namespace ppo

#define PPO_RCCL_API(api)                                                   \
  const ppo::RcclApi *api = ppo::rccl();                                    \
  if (!api) {                                                               \
    ppo::set_error("%s", ppo::g_rccl.err);                                  \
    return PPO_EHIP;                                                        \
  }

#define PPO_NCCL_TRY(api, call)                                                      \
  do {                                                                               \
    ncclResult_t r_ = (call);                                                        \
    if (r_ != ncclSuccess) {                                                         \
      ppo::set_error("%s failed: %s", #call, api->error_string(r_));                 \
      return PPO_EHIP;                                                               \
    }                                                                                \
  } while (0)

extern "C" int ppo_comm_version(void) {
  const ppo::RcclApi *api = ppo::rccl();
  int v = 0;
  if (!api || api->get_version(&v) != ncclSuccess) return 0;
  return v;
}

extern "C" int ppo_comm_unique_id(uint8_t *id_out) {
  PPO_REQUIRE(id_out != nullptr, "ppo_comm_unique_id: null output");
  PPO_RCCL_API(api);
  ncclUniqueId id;
  PPO_NCCL_TRY(api, api->get_unique_id(&id));
  static_assert(sizeof(id) == PPO_COMM_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id_out, &id, sizeof(id));
  return 0;
}

extern "C" int ppo_comm_create(const uint8_t *id, int nranks, int rank, int device,
                               ppo_comm **out) {
  PPO_REQUIRE(id != nullptr && out != nullptr, "ppo_comm_create: null argument");
  PPO_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "ppo_comm_create: rank %d of %d", rank,
              nranks);
  *out = nullptr;
  PPO_RCCL_API(api);
  PPO_HIP_TRY(hipSetDevice(device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ppo_comm *c = new (std::nothrow) ppo_comm();
  PPO_REQUIRE(c != nullptr, "ppo_comm_create: out of host memory");
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  const ncclResult_t r = api->comm_init_rank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    ppo::set_error("ncclCommInitRank(%d of %d) failed: %s", rank, nranks, api->error_string(r));
    delete c;
    return PPO_EHIP;
  }
  *out = c;
  return 0;
}

extern "C" int ppo_comm_destroy(ppo_comm *c) {
  if (!c) return 0;
  const ppo::RcclApi *api = ppo::rccl();
  if (api) (void)api->comm_destroy(c->comm);
  delete c;
  return 0;
}

extern "C" int ppo_comm_allreduce(ppo_comm *c, float *buf_d, int64_t n, void *stream) {
  PPO_REQUIRE(c != nullptr && buf_d != nullptr && n >= 0, "ppo_comm_allreduce: bad argument");
  PPO_RCCL_API(api);
  if (n == 0) return 0;
  // in place (sendbuff == recvbuff), SUM over the communicator, ordered on the caller's stream:
  // legal inside a hipGraph capture of that stream
  PPO_NCCL_TRY(api, api->all_reduce(buf_d, buf_d, static_cast<size_t>(n), ncclFloat32, ncclSum,
                                    c->comm, ppo::as_stream(stream)));
  return 0;
}

extern "C" int ppo_comm_check(ppo_comm *c) {
  PPO_REQUIRE(c != nullptr, "ppo_comm_check: null comm");
  PPO_RCCL_API(api);
  ncclResult_t async = ncclSuccess;
  PPO_NCCL_TRY(api, api->async_error(c->comm, &async));
  if (async != ncclSuccess && async != ncclInProgress) {
    ppo::set_error("RCCL asynchronous error: %s", api->error_string(async));
    return PPO_EHIP;
  }
  return 0;
}

// The communicator's own view (not the arguments it was created with): RCCL's rank count and
// this rank, plus the device -- what the bench line reports as "comm".
extern "C" int ppo_comm_query(ppo_comm *c, int *nranks_out, int *rank_out, int *device_out) {
  PPO_REQUIRE(c != nullptr, "ppo_comm_query: null comm");
  PPO_RCCL_API(api);
  int n = 0, r = -1;
  PPO_NCCL_TRY(api, api->comm_count(c->comm, &n));
  PPO_NCCL_TRY(api, api->comm_user_rank(c->comm, &r));
  if (nranks_out) *nranks_out = n;
  if (rank_out) *rank_out = r;
  if (device_out) *device_out = c->device;
  return 0;
}

// SURVEY.md s8(b)'s ppo_allreduce_grads(ctx, flat, n, stream): the ctx's attached communicator.
extern "C" int ppo_ctx_set_comm(ppo_ctx *ctx, ppo_comm *c) {
  PPO_REQUIRE(ctx != nullptr, "ppo_ctx_set_comm: null ctx");
  PPO_REQUIRE(c == nullptr || c->device == ctx->device,
              "ppo_ctx_set_comm: communicator on device %d, ctx on %d", c ? c->device : -1,
              ctx->device);
  ctx->comm = c;
  return 0;
}

extern "C" int ppo_allreduce_grads(ppo_ctx *ctx, float *flat_d, int64_t n, void *stream) {
  PPO_REQUIRE(ctx != nullptr, "ppo_allreduce_grads: null ctx");
  PPO_REQUIRE(ctx->comm != nullptr, "ppo_allreduce_grads: no communicator (ppo_ctx_set_comm)");
  PPO_REQUIRE(n >= 0 && n <= ctx->total_params,
              "ppo_allreduce_grads: %lld floats, the flat layout holds %lld",
              static_cast<long long>(n), static_cast<long long>(ctx->total_params));
  return ppo_comm_allreduce(ctx->comm, flat_d, n, stream);
}
