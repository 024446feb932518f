// Native RCCL communicator (SURVEY.md §5.8 data plane): collectives issued on the
// caller's HIP stream with raw device pointers, over xGMI between the GPUs of a node.
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <vector>

struct ncclComm;

namespace atpu {

class RcclComm {
 public:
  // ncclCommInitRank on `device` (this process's GPU); `uid` from unique_id() on one rank
  RcclComm(int world, int rank, const std::string& uid, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  static std::string unique_id();
  // single-process communicators over several local GPUs (ncclCommInitAll)
  static std::vector<std::shared_ptr<RcclComm>> init_all(const std::vector<int>& devices);

  // dtype: 0 int8, 1 uint8, 2 int32, 4 int64, 7 fp32, 8 fp64, 9 bf16 (ncclDataType_t values)
  void broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s);
  void all_gather(const void* send, void* recv, size_t count_per_rank, int dtype, hipStream_t s);
  // op: 0 sum, 1 prod, 2 max, 3 min (ncclRedOp_t values)
  void all_reduce(void* buf, size_t count, int dtype, int op, hipStream_t s);
  // 0 = healthy; otherwise the communicator's asynchronous error (a peer failed)
  int async_error() const;
  void abort();

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }

 private:
  RcclComm() = default;
  ncclComm* comm_ = nullptr;
  int rank_ = 0, world_ = 1, device_ = 0;
};

void rccl_group_start();
void rccl_group_end();
int rccl_version();

}  // namespace atpu
