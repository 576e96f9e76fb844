// Test stand-in for <hip/hip_runtime.h>: just the host API lmpc_multi.cpp calls, over host memory, so that the
// library's shard / scatter / gather bookkeeping compiles and runs on a CPU (tests/cpp/multi_shard_test.cpp).
// Never used by the product build (liblmpc_multi.so links the real HIP runtime and librccl).
#pragma once
#include <cstddef>

typedef int hipError_t;
typedef struct ihipStream_t* hipStream_t;
enum { hipSuccess = 0, hipErrorOutOfMemory = 2 };
enum hipMemcpyKind { hipMemcpyHostToHost, hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice };
constexpr unsigned hipStreamNonBlocking = 1;

hipError_t hipGetDevice(int* d);
hipError_t hipSetDevice(int d);
hipError_t hipGetDeviceCount(int* n);
hipError_t hipMalloc(void** p, size_t bytes);
template <class T>
inline hipError_t hipMalloc(T** p, size_t bytes) { return hipMalloc(reinterpret_cast<void**>(p), bytes); }
hipError_t hipFree(void* p);
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned flags);
hipError_t hipStreamDestroy(hipStream_t s);
hipError_t hipStreamSynchronize(hipStream_t s);
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s);
