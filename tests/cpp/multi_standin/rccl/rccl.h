// Test stand-in for <rccl/rccl.h>: the six calls lmpc_multi.cpp makes (ncclCommInitAll, ncclCommDestroy,
// ncclGroupStart / ncclGroupEnd, ncclSend / ncclRecv), backed by memcpy between host buffers.  A group records its
// sends and receives and, at ncclGroupEnd, matches every receive to the send between the same pair of ranks (in
// issue order), checks type and count agree, and copies.  Any unmatched or mismatched call fails the group.
#pragma once
#include <cstddef>

typedef enum { ncclSuccess = 0, ncclInvalidUsage = 5 } ncclResult_t;
typedef enum { ncclInt8 = 0, ncclUint8 = 1, ncclInt32 = 2, ncclUint32 = 3, ncclInt64 = 4, ncclUint64 = 5,
               ncclFloat16 = 6, ncclFloat32 = 7, ncclFloat64 = 8 } ncclDataType_t;
typedef struct ncclComm* ncclComm_t;
typedef struct ihipStream_t* hipStream_t;

ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist);
ncclResult_t ncclCommDestroy(ncclComm_t comm);
ncclResult_t ncclGroupStart();
ncclResult_t ncclGroupEnd();
ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm, hipStream_t s);
ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm, hipStream_t s);
