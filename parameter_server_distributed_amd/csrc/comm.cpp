#include "comm.h"

#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <rccl/rccl.h>

#include <cstring>

namespace psd {

namespace {

#define RCCL_CHECK(expr)                                                                           \
  do {                                                                                             \
    ncclResult_t _r = (expr);                                                                      \
    TORCH_CHECK(_r == ncclSuccess, "psd rccl: ", #expr, " failed: ", ncclGetErrorString(_r));      \
  } while (0)

ncclDataType_t nccl_type(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    case at::kFloat8_e4m3fn: return ncclFloat8e4m3;
    default: TORCH_CHECK(false, "psd rccl: unsupported dtype ", t.scalar_type());
  }
}

ncclRedOp_t nccl_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "avg") return ncclAvg;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  TORCH_CHECK(false, "psd rccl: unknown reduce op ", op);
}

hipStream_t pick_stream(const at::Tensor& t, int64_t stream) {
  if (stream != 0) return reinterpret_cast<hipStream_t>(stream);
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void need_cuda(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "psd rccl: tensors must be contiguous device tensors");
}

}  // namespace

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

int RcclComm::version() {
  int v = 0;
  RCCL_CHECK(ncclGetVersion(&v));
  return v;
}

RcclComm::RcclComm(int rank, int world, const std::string& uid, int device)
    : rank_(rank), world_(world), device_(device) {
  TORCH_CHECK(uid.size() == NCCL_UNIQUE_ID_BYTES, "psd rccl: unique id must be 128 bytes");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  const c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  ncclComm_t c = nullptr;
  RCCL_CHECK(ncclCommInitRank(&c, world, id, rank));
  comm_ = c;
}

RcclComm::~RcclComm() {
  if (comm_) {
    ncclCommDestroy(static_cast<ncclComm_t>(comm_));
    comm_ = nullptr;
  }
}

void RcclComm::abort() {
  if (comm_) {
    ncclCommAbort(static_cast<ncclComm_t>(comm_));
    comm_ = nullptr;
  }
}

std::string RcclComm::async_error() {
  if (!comm_) return "aborted";
  ncclResult_t e = ncclSuccess;
  RCCL_CHECK(ncclCommGetAsyncError(static_cast<ncclComm_t>(comm_), &e));
  return e == ncclSuccess ? std::string() : std::string(ncclGetErrorString(e));
}

#define COMM static_cast<ncclComm_t>(comm_)

void RcclComm::all_reduce(at::Tensor t, const std::string& op, int64_t stream) {
  need_cuda(t);
  TORCH_CHECK(comm_, "psd rccl: communicator aborted");
  RCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_type(t), nccl_op(op), COMM, pick_stream(t, stream)));
}

void RcclComm::reduce_scatter(const at::Tensor& in, at::Tensor out, const std::string& op, int64_t stream) {
  need_cuda(in);
  need_cuda(out);
  TORCH_CHECK(in.numel() == out.numel() * world_, "psd rccl: reduce_scatter needs in.numel == world * out.numel");
  RCCL_CHECK(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), nccl_type(in), nccl_op(op), COMM,
                               pick_stream(in, stream)));
}

void RcclComm::all_gather(const at::Tensor& in, at::Tensor out, int64_t stream) {
  need_cuda(in);
  need_cuda(out);
  TORCH_CHECK(out.numel() == in.numel() * world_, "psd rccl: all_gather needs out.numel == world * in.numel");
  RCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), nccl_type(in), COMM, pick_stream(in, stream)));
}

void RcclComm::reduce(const at::Tensor& in, at::Tensor out, int root, const std::string& op, int64_t stream) {
  need_cuda(in);
  need_cuda(out);
  RCCL_CHECK(ncclReduce(in.data_ptr(), out.data_ptr(), in.numel(), nccl_type(in), nccl_op(op), root, COMM,
                        pick_stream(in, stream)));
}

void RcclComm::broadcast(at::Tensor t, int root, int64_t stream) {
  need_cuda(t);
  RCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_type(t), root, COMM, pick_stream(t, stream)));
}

void RcclComm::send(const at::Tensor& t, int peer, int64_t stream) {
  need_cuda(t);
  RCCL_CHECK(ncclSend(t.data_ptr(), t.numel(), nccl_type(t), peer, COMM, pick_stream(t, stream)));
}

void RcclComm::recv(at::Tensor t, int peer, int64_t stream) {
  need_cuda(t);
  RCCL_CHECK(ncclRecv(t.data_ptr(), t.numel(), nccl_type(t), peer, COMM, pick_stream(t, stream)));
}

void RcclComm::group_start() { RCCL_CHECK(ncclGroupStart()); }
void RcclComm::group_end() { RCCL_CHECK(ncclGroupEnd()); }

#undef COMM

}  // namespace psd
