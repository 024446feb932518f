// Native RCCL communicator (C1 weight broadcast, C2 row all-gather,
// C3 risk all-reduce of §2.7). The DP layer (agent_tpu_amd/parallel/dp.py) issues
// its collectives through torch.distributed by default; ATPU_COMM=native routes the
// data-plane collectives here instead: raw device pointers on the caller's HIP
// stream, no tensor wrapping, and the single-process multi-GPU form (ncclCommInitAll)
// SURVEY §5.8 recommends for an agent that owns every GPU of the node.
#include "atpu/comm.h"

#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>

#include "atpu/common.h"

namespace atpu {
namespace {

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}

ncclDataType_t dt(int d) {
  switch (d) {
    case 0: return ncclInt8;
    case 1: return ncclUint8;
    case 2: return ncclInt32;
    case 4: return ncclInt64;
    case 7: return ncclFloat32;
    case 8: return ncclFloat64;
    case 9: return ncclBfloat16;
    default: throw std::invalid_argument("rccl: unsupported dtype code " + std::to_string(d));
  }
}

ncclRedOp_t rop(int o) {
  switch (o) {
    case 0: return ncclSum;
    case 1: return ncclProd;
    case 2: return ncclMax;
    case 3: return ncclMin;
    default: throw std::invalid_argument("rccl: unsupported reduction " + std::to_string(o));
  }
}

struct DeviceGuard {
  int prev = 0;
  explicit DeviceGuard(int d) {
    ATPU_HIP_CHECK(hipGetDevice(&prev));
    if (prev != d) ATPU_HIP_CHECK(hipSetDevice(d));
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

}  // namespace

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

RcclComm::RcclComm(int world, int rank, const std::string& uid, int device)
    : rank_(rank), world_(world), device_(device) {
  ATPU_CHECK(world >= 1 && rank >= 0 && rank < world, "rccl: bad rank / world");
  ATPU_CHECK(uid.size() == sizeof(ncclUniqueId), "rccl: unique id must be NCCL_UNIQUE_ID_BYTES long");
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  DeviceGuard g(device);
  ncclComm_t c = nullptr;
  check(ncclCommInitRank(&c, world, id, rank), "ncclCommInitRank");
  comm_ = c;
}

std::vector<std::shared_ptr<RcclComm>> RcclComm::init_all(const std::vector<int>& devices) {
  ATPU_CHECK(!devices.empty(), "rccl: no devices");
  std::vector<ncclComm_t> cs(devices.size(), nullptr);
  check(ncclCommInitAll(cs.data(), static_cast<int>(devices.size()), devices.data()), "ncclCommInitAll");
  std::vector<std::shared_ptr<RcclComm>> out;
  for (size_t i = 0; i < devices.size(); ++i) {
    std::shared_ptr<RcclComm> c(new RcclComm());
    c->comm_ = cs[i];
    c->rank_ = static_cast<int>(i);
    c->world_ = static_cast<int>(devices.size());
    c->device_ = devices[i];
    out.push_back(c);
  }
  return out;
}

RcclComm::~RcclComm() {
  if (comm_) (void)ncclCommDestroy(comm_);
}

void RcclComm::abort() {
  if (comm_) {
    (void)ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

int RcclComm::async_error() const {
  if (!comm_) return -1;
  ncclResult_t e = ncclSuccess;
  if (ncclCommGetAsyncError(comm_, &e) != ncclSuccess) return -1;
  return static_cast<int>(e);
}

void RcclComm::broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s) {
  ATPU_CHECK(comm_, "rccl: communicator aborted");
  DeviceGuard g(device_);
  check(ncclBroadcast(buf, buf, count, dt(dtype), root, comm_, s), "ncclBroadcast");
}

void RcclComm::all_gather(const void* send, void* recv, size_t count_per_rank, int dtype, hipStream_t s) {
  ATPU_CHECK(comm_, "rccl: communicator aborted");
  DeviceGuard g(device_);
  check(ncclAllGather(send, recv, count_per_rank, dt(dtype), comm_, s), "ncclAllGather");
}

void RcclComm::all_reduce(void* buf, size_t count, int dtype, int op, hipStream_t s) {
  ATPU_CHECK(comm_, "rccl: communicator aborted");
  DeviceGuard g(device_);
  check(ncclAllReduce(buf, buf, count, dt(dtype), rop(op), comm_, s), "ncclAllReduce");
}

void rccl_group_start() { check(ncclGroupStart(), "ncclGroupStart"); }
void rccl_group_end() { check(ncclGroupEnd(), "ncclGroupEnd"); }

int rccl_version() {
  int v = 0;
  check(ncclGetVersion(&v), "ncclGetVersion");
  return v;
}

}  // namespace atpu
