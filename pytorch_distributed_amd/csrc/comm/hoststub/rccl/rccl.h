// Host-only stand-in for the RCCL (NCCL 2.x) API subset csrc/comm uses. The implementation
// (stub_runtime.cpp) runs every collective synchronously on host memory across the threads that
// hold the ranks of one communicator, so the C++ reducer can be exercised with world > 1 under
// the sanitizers on a machine without GPUs. Test-only (see hip/hip_runtime.h beside it).
#pragma once

#include <cstddef>

#include "../hip/hip_runtime.h"

#define NCCL_UNIQUE_ID_BYTES 128

typedef enum {
  ncclSuccess = 0,
  ncclUnhandledCudaError = 1,
  ncclSystemError = 2,
  ncclInternalError = 3,
  ncclInvalidArgument = 4,
  ncclInvalidUsage = 5,
  ncclRemoteError = 6,
  ncclInProgress = 7,
  ncclNumResults = 8
} ncclResult_t;

typedef enum {
  ncclInt8 = 0, ncclUint8 = 1, ncclInt32 = 2, ncclUint32 = 3, ncclInt64 = 4, ncclUint64 = 5,
  ncclFloat16 = 6, ncclFloat32 = 7, ncclFloat64 = 8, ncclBfloat16 = 9
} ncclDataType_t;

typedef enum { ncclSum = 0, ncclProd = 1, ncclMax = 2, ncclMin = 3, ncclAvg = 4 } ncclRedOp_t;

typedef struct { char internal[NCCL_UNIQUE_ID_BYTES]; } ncclUniqueId;

struct pda_stub_comm;
typedef pda_stub_comm* ncclComm_t;

ncclResult_t ncclGetUniqueId(ncclUniqueId* id);
const char* ncclGetErrorString(ncclResult_t r);
ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank);
ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist);
ncclResult_t ncclCommDestroy(ncclComm_t comm);
ncclResult_t ncclCommAbort(ncclComm_t comm);
ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* err);
ncclResult_t ncclCommCount(ncclComm_t comm, int* count);
ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, ncclDataType_t dt,
                           ncclRedOp_t op, ncclComm_t comm, hipStream_t st);
ncclResult_t ncclBroadcast(const void* send, void* recv, size_t count, ncclDataType_t dt, int root,
                           ncclComm_t comm, hipStream_t st);
ncclResult_t ncclReduce(const void* send, void* recv, size_t count, ncclDataType_t dt,
                        ncclRedOp_t op, int root, ncclComm_t comm, hipStream_t st);
ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t dt,
                           ncclComm_t comm, hipStream_t st);
ncclResult_t ncclReduceScatter(const void* send, void* recv, size_t count, ncclDataType_t dt,
                               ncclRedOp_t op, ncclComm_t comm, hipStream_t st);
ncclResult_t ncclGroupStart();
ncclResult_t ncclGroupEnd();

// test hooks (stub only)
extern "C" void pda_stub_inject_async_error(ncclComm_t comm);
extern "C" long pda_stub_collectives(void);
