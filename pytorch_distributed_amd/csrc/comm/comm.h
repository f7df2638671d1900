// Shared between the RCCL communicator (rccl_comm.cpp) and the gradient-bucket reducer
// (reducer.cpp): the communicator handle handed to Python as an opaque pointer.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <vector>

namespace pda {

struct Comm {
  std::vector<ncclComm_t> comms;  // 1 for multi-process, ndev for in-process
  std::vector<int> devices;
};

inline ncclDataType_t to_nccl(int dt) {
  switch (dt) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclInt64;
    case 4: return ncclFloat64;
    case 5: return ncclInt32;
    default: return ncclFloat32;
  }
}

inline size_t nccl_elem_bytes(int dt) {
  switch (dt) {
    case 1: case 2: return 2;
    case 3: case 4: return 8;
    default: return 4;
  }
}

}  // namespace pda
