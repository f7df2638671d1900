// Host-only stand-in for the few HIP runtime calls csrc/comm uses, so the communicator and the
// gradient-bucket reducer compile with g++ and run under AddressSanitizer / ThreadSanitizer on the
// CPU. Test-only: never on the include path of the real build (_build.py).
#pragma once

#include <cstddef>

typedef enum hipError_t { hipSuccess = 0, hipErrorInvalidValue = 1, hipErrorNotReady = 600 } hipError_t;

struct pda_stub_stream;
struct pda_stub_event;
typedef pda_stub_stream* hipStream_t;
typedef pda_stub_event* hipEvent_t;

#define hipEventDefault 0x0
#define hipEventDisableTiming 0x2

hipError_t hipSetDevice(int device);
hipError_t hipEventCreate(hipEvent_t* e);
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned flags);
hipError_t hipEventDestroy(hipEvent_t e);
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s);
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned flags);
hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b);
