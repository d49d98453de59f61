// comm.hip — posterior pooling across GPUs over RCCL (the C-ABI half of SURVEY §8e).
//
// The reference runs chains on a process pool and concatenates the per-process posterior
// DataFrames (Framework.py:779-780 Pool.starmap, :1037 pd.concat).  Here every rank holds
// its walkers' sample block [rows][count_r] (walker-minor, the oe_mh_run layout) in HBM
// and ONE ncclAllGather over xGMI pools them; the rank-major result is then laid out as
// [rows][n_total] in global walker order with one strided copy per rank.
//
// RCCL is opened at run time (dlopen "librccl.so", the name PyTorch's ROCm build links,
// so a process that already has torch's RCCL shares that instance; then "librccl.so.1"
// from the library's runpath): the engine does not need RCCL unless pooling is used.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/odelib_amd.h"

namespace {

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  std::string err;
};

Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    for (const char* name : {"librccl.so", "librccl.so.1"}) {
      x.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
      if (x.h) break;
    }
    if (!x.h) {
      const char* e = dlerror();
      x.err = std::string("RCCL not available: ") + (e ? e : "dlopen failed");
      return x;
    }
    x.get_unique_id = reinterpret_cast<decltype(x.get_unique_id)>(dlsym(x.h, "ncclGetUniqueId"));
    x.comm_init_rank = reinterpret_cast<decltype(x.comm_init_rank)>(dlsym(x.h, "ncclCommInitRank"));
    x.comm_destroy = reinterpret_cast<decltype(x.comm_destroy)>(dlsym(x.h, "ncclCommDestroy"));
    x.all_gather = reinterpret_cast<decltype(x.all_gather)>(dlsym(x.h, "ncclAllGather"));
    x.error_string = reinterpret_cast<decltype(x.error_string)>(dlsym(x.h, "ncclGetErrorString"));
    if (!x.get_unique_id || !x.comm_init_rank || !x.comm_destroy || !x.all_gather || !x.error_string)
      x.err = "RCCL library lacks ncclGetUniqueId / ncclCommInitRank / ncclAllGather";
    return x;
  }();
  return r;
}

thread_local std::string g_comm_err;

int comm_fail(oe_comm* c, int code, const std::string& msg);

}  // namespace

struct oe_comm {
  ncclComm_t nc = nullptr;
  int32_t n_ranks = 0, rank = 0, device = 0;
  hipStream_t stream = nullptr;  // launch stream of the collective (oe_comm_set_stream; null = legacy)
  void* stage = nullptr;         // padded send block and rank-major receive buffer
  size_t stage_bytes = 0;
  std::string err;
};

namespace {

int comm_fail(oe_comm* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  else g_comm_err = msg;
  return code;
}

#define OE_NCCL(c, expr)                                                                          \
  do {                                                                                            \
    ncclResult_t r_ = (expr);                                                                     \
    if (r_ != ncclSuccess) return comm_fail(c, OE_ERR_HIP, std::string(#expr) + ": " + R.error_string(r_)); \
  } while (0)
#define OE_HIPC(c, expr)                                                                          \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) return comm_fail(c, OE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct DevGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DevGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) err = hipSetDevice(d);
    else prev = -1;
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// the data movement around the collective, usable without a communicator
// (oe_pool_pad / oe_pool_relayout): one rank's block padded to [rows][cmax] ...
hipError_t pad_block(int64_t rows, const double* block, int64_t cnt, int64_t cmax, double* padded, hipStream_t s) {
  hipError_t e = hipMemsetAsync(padded, 0, sizeof(double) * (size_t)rows * (size_t)cmax, s);
  if (e != hipSuccess || cnt == 0) return e;
  return hipMemcpy2DAsync(padded, sizeof(double) * cmax, block, sizeof(double) * cnt, sizeof(double) * cnt,
                          (size_t)rows, hipMemcpyDeviceToDevice, s);
}

// ... and the gathered rank-major [n][rows][cmax] laid out walker-minor [rows][n_total] in
// global walker order (rank r's walkers at columns off[r] .. off[r] + counts[r]): one strided
// copy per rank
hipError_t relayout(int n, int64_t rows, const int64_t* counts, const int64_t* off, int64_t cmax,
                    const double* gathered, double* out, hipStream_t s) {
  for (int r = 0; r < n; ++r) {
    if (counts[r] == 0) continue;
    const hipError_t e = hipMemcpy2DAsync(out + off[r], sizeof(double) * off[n], gathered + (size_t)r * rows * cmax,
                                          sizeof(double) * cmax, sizeof(double) * counts[r], (size_t)rows,
                                          hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

extern "C" {

int oe_pool_pad(int64_t rows, const double* block, int64_t count, int64_t cmax, double* padded, void* hip_stream,
                uint32_t flags) {
  if (rows < 0 || count < 0 || cmax < count || (rows > 0 && cmax > 0 && !padded) || (rows > 0 && count > 0 && !block))
    return comm_fail(nullptr, OE_ERR_ARG, "oe_pool_pad: need 0 <= count <= cmax and device buffers");
  if (rows == 0 || cmax == 0) return OE_OK;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  OE_HIPC(nullptr, pad_block(rows, block, count, cmax, padded, s));
  if (!(flags & OE_ASYNC)) OE_HIPC(nullptr, hipStreamSynchronize(s));
  return OE_OK;
}

int oe_pool_relayout(int32_t n_ranks, int64_t rows, const int64_t* counts, const double* gathered, double* out,
                     void* hip_stream, uint32_t flags) {
  if (n_ranks < 1 || rows < 0 || !counts) return comm_fail(nullptr, OE_ERR_ARG, "oe_pool_relayout: bad arguments");
  std::vector<int64_t> off(n_ranks + 1, 0);
  int64_t cmax = 0;
  for (int r = 0; r < n_ranks; ++r) {
    if (counts[r] < 0) return comm_fail(nullptr, OE_ERR_ARG, "oe_pool_relayout: negative count");
    off[r + 1] = off[r] + counts[r];
    cmax = std::max(cmax, counts[r]);
  }
  if (rows == 0 || cmax == 0) return OE_OK;
  if (!gathered || !out) return comm_fail(nullptr, OE_ERR_ARG, "oe_pool_relayout: null buffer");
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  OE_HIPC(nullptr, relayout(n_ranks, rows, counts, off.data(), cmax, gathered, out, s));
  if (!(flags & OE_ASYNC)) OE_HIPC(nullptr, hipStreamSynchronize(s));
  return OE_OK;
}

int oe_comm_unique_id(uint8_t* id, int32_t id_bytes) {
  if (!id || id_bytes != OE_COMM_ID_BYTES) return comm_fail(nullptr, OE_ERR_ARG, "oe_comm_unique_id: need a 128-byte buffer");
  Rccl& R = rccl();
  if (!R.err.empty()) return comm_fail(nullptr, OE_ERR_UNSUPPORTED, R.err);
  ncclUniqueId u;
  OE_NCCL(nullptr, R.get_unique_id(&u));
  std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return OE_OK;
}

int oe_comm_init(int32_t device, int32_t n_ranks, int32_t rank, const uint8_t* id, int32_t id_bytes, oe_comm** out) {
  if (!out) return comm_fail(nullptr, OE_ERR_ARG, "oe_comm_init: null out");
  *out = nullptr;
  if (!id || id_bytes != OE_COMM_ID_BYTES || n_ranks < 1 || rank < 0 || rank >= n_ranks)
    return comm_fail(nullptr, OE_ERR_ARG, "oe_comm_init: need 0 <= rank < n_ranks and a 128-byte id");
  Rccl& R = rccl();
  if (!R.err.empty()) return comm_fail(nullptr, OE_ERR_UNSUPPORTED, R.err);
  DevGuard g(device);
  if (g.err != hipSuccess) return comm_fail(nullptr, OE_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(g.err));
  oe_comm* c = new (std::nothrow) oe_comm();
  if (!c) return OE_ERR_NOMEM;
  ncclUniqueId u;
  std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  const ncclResult_t r = R.comm_init_rank(&c->nc, n_ranks, u, rank);
  if (r != ncclSuccess) {
    const std::string msg = std::string("ncclCommInitRank: ") + R.error_string(r);
    delete c;
    return comm_fail(nullptr, OE_ERR_HIP, msg);
  }
  c->n_ranks = n_ranks;
  c->rank = rank;
  c->device = device;
  *out = c;
  return OE_OK;
}

void oe_comm_destroy(oe_comm* c) {
  if (!c) return;
  DevGuard g(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  else (void)hipDeviceSynchronize();
  if (c->stage) (void)hipFree(c->stage);
  if (c->nc) (void)rccl().comm_destroy(c->nc);
  delete c;
}

const char* oe_comm_last_error(const oe_comm* c) {
  if (c) return c->err.c_str();
  return g_comm_err.empty() ? "null communicator" : g_comm_err.c_str();
}

int oe_comm_set_stream(oe_comm* c, void* hip_stream) {
  if (!c) return OE_ERR_ARG;
  c->stream = static_cast<hipStream_t>(hip_stream);
  return OE_OK;
}

int oe_allgather_samples(oe_comm* c, int64_t rows, const double* block, const int64_t* counts, double* out,
                         uint32_t flags) {
  if (!c) return comm_fail(nullptr, OE_ERR_ARG, "oe_allgather_samples: null communicator");
  if (rows < 0 || !counts || (rows > 0 && !out)) return comm_fail(c, OE_ERR_ARG, "oe_allgather_samples: bad arguments");
  if (flags & OE_HOST_PTRS) return comm_fail(c, OE_ERR_ARG, "oe_allgather_samples: device pointers only");
  Rccl& R = rccl();
  const int n = c->n_ranks;
  std::vector<int64_t> off(n + 1, 0);
  int64_t cmax = 0;
  for (int r = 0; r < n; ++r) {
    if (counts[r] < 0) return comm_fail(c, OE_ERR_ARG, "oe_allgather_samples: negative count");
    off[r + 1] = off[r] + counts[r];
    cmax = std::max(cmax, counts[r]);
  }
  const int64_t cnt = counts[c->rank];
  if (rows == 0 || cmax == 0) return OE_OK;
  if (cnt > 0 && !block) return comm_fail(c, OE_ERR_ARG, "oe_allgather_samples: null block");
  DevGuard g(c->device);
  if (g.err != hipSuccess) return comm_fail(c, OE_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(g.err));
  hipStream_t s = c->stream;
  const size_t blk = sizeof(double) * (size_t)rows * (size_t)cmax;  // one rank's padded block
  // every rank's block, padded to [rows][cmax], lands rank-major in a staging buffer and is
  // re-laid walker-minor into out; n == 1 gathers straight into out
  const size_t need = (n == 1 ? 0 : blk * (size_t)n) + (cnt < cmax ? blk : 0);
  if (c->stage_bytes < need) {
    if (c->stage) {
      OE_HIPC(c, hipStreamSynchronize(s));
      OE_HIPC(c, hipFree(c->stage));
      c->stage = nullptr;
      c->stage_bytes = 0;
    }
    OE_HIPC(c, hipMalloc(&c->stage, need));
    c->stage_bytes = need;
  }
  char* base = static_cast<char*>(c->stage);
  double* gathered = n == 1 ? out : reinterpret_cast<double*>(base);
  const double* send = block;
  if (cnt < cmax) {  // pad this rank's block to [rows][cmax]
    double* pad = reinterpret_cast<double*>(base + (n == 1 ? 0 : blk * (size_t)n));
    OE_HIPC(c, pad_block(rows, block, cnt, cmax, pad, s));
    send = pad;
  }
  OE_NCCL(c, R.all_gather(send, gathered, (size_t)rows * (size_t)cmax, ncclFloat64, c->nc, s));
  // rank-major [n][rows][cmax] -> walker-minor [rows][n_total], rank r at column off[r]
  if (n > 1) OE_HIPC(c, relayout(n, rows, counts, off.data(), cmax, gathered, out, s));
  if (!(flags & OE_ASYNC)) OE_HIPC(c, hipStreamSynchronize(s));
  return OE_OK;
}

}  // extern "C"
