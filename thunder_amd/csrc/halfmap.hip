// halfmap.hip -- a13: the per-hemisphere half-map reduction over RCCL.
//
// The reference sums every GPU's partial F3D / T3D / O3D / counter of one
// gold-standard hemisphere inside cuthunder::InsertFT: ncclGetUniqueId on the
// hemisphere's first rank, MPI_Bcast of the id over `hemi`, ncclCommInitRank
// over (ranks x local GPUs) (gpu/src/cuthunder.cu:5294-5324), then in-place
// ncclAllReduce of F (2 dimSize floats), T (dimSize floats), O (3 doubles)
// and counter (gpu/src/cuthunder.cu:5903-5993).  Here the same exchange is a
// C-ABI call on a caller-owned communicator -- one process per GPU, so the
// communicator spans the hemisphere's ranks; the id travels over whatever the
// host uses (MPI_Bcast in a C++/MPI THUNDER host, torch.distributed in
// bench.py).  The counter is reduced as int32 (the reference passes a 4-byte
// int as ncclInt64, quirk q2).  RCCL runs over xGMI between the GPUs of one
// node; the four collectives are one ncclGroup so RCCL can schedule them
// together.
#include <rccl/rccl.h>

#include <cstring>

#include "common.h"

#define THX_NCCL(call)                                                         \
    do {                                                                       \
        ncclResult_t r_ = (call);                                              \
        if (r_ != ncclSuccess) {                                               \
            ::thx::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call,        \
                             ncclGetErrorString(r_));                          \
            return THX_ERR_HIP;                                                \
        }                                                                      \
    } while (0)

static_assert(NCCL_UNIQUE_ID_BYTES == THX_RCCL_ID_BYTES, "unique-id size");

extern "C" int thx_rccl_unique_id(void* id)
{
    THX_CHECK_ARG(id, "thx_rccl_unique_id: null");
    ncclUniqueId u;
    THX_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return THX_OK;
}

extern "C" int thx_rccl_comm_init(int nranks, const void* id, int rank, void** comm)
{
    THX_CHECK_ARG(id && comm && nranks > 0 && rank >= 0 && rank < nranks,
                  "thx_rccl_comm_init: bad arguments");
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    THX_NCCL(ncclCommInitRank(&c, nranks, u, rank));
    *comm = c;
    return THX_OK;
}

extern "C" int thx_rccl_comm_destroy(void* comm)
{
    if (comm) THX_NCCL(ncclCommDestroy(static_cast<ncclComm_t>(comm)));
    return THX_OK;
}

// Inside a group the first failure is kept and the group is still closed, so
// the calling thread never keeps an open ncclGroup after an error.
#define THX_NCCL_GROUPED(call)                                                 \
    do {                                                                       \
        ncclResult_t r_ = (call);                                              \
        if (r_ != ncclSuccess && first == ncclSuccess) {                       \
            first = r_;                                                        \
            what = #call;                                                      \
        }                                                                      \
    } while (0)

static int group_end(ncclResult_t first, const char* what)
{
    const ncclResult_t e = ncclGroupEnd();
    if (first == ncclSuccess && e != ncclSuccess) {
        first = e;
        what = "ncclGroupEnd()";
    }
    if (first != ncclSuccess) {
        ::thx::set_error("halfmap.hip %s: %s", what, ncclGetErrorString(first));
        return THX_ERR_HIP;
    }
    return THX_OK;
}

namespace thx {
int comm_device(void* comm, int* dev)
{
    THX_CHECK_ARG(comm && dev, "comm_device: null");
    THX_NCCL(ncclCommCuDevice(static_cast<ncclComm_t>(comm), dev));
    return THX_OK;
}

// oDim doubles of O per class (3 in 3D, 2 for the 2D InsertI2D's O2D)
int halfmap_allreduce_impl(void* comm, float* F, float* T, double* O, int oDim, int* counter,
                           long long dimSize, int nK, hipStream_t s)
{
    THX_CHECK_ARG(comm && F && T && dimSize > 0 && nK >= 1 && oDim > 0,
                  "thx_halfmap_allreduce: bad arguments");
    ncclComm_t c = static_cast<ncclComm_t>(comm);
    const size_t n = (size_t)dimSize * nK;
    THX_NCCL(ncclGroupStart());
    ncclResult_t first = ncclSuccess;
    const char* what = "";
    THX_NCCL_GROUPED(ncclAllReduce(F, F, 2 * n, ncclFloat32, ncclSum, c, s));
    THX_NCCL_GROUPED(ncclAllReduce(T, T, n, ncclFloat32, ncclSum, c, s));
    if (O) THX_NCCL_GROUPED(ncclAllReduce(O, O, (size_t)oDim * nK, ncclFloat64, ncclSum, c, s));
    if (counter) THX_NCCL_GROUPED(ncclAllReduce(counter, counter, nK, ncclInt32, ncclSum, c, s));
    return group_end(first, what);
}
}  // namespace thx

extern "C" int thx_halfmap_allreduce(void* comm, float* F, float* T, double* O, int* counter,
                                     long long dimSize, int nK, thx_stream_t stream)
{
    return thx::halfmap_allreduce_impl(comm, F, T, O, 3, counter, dimSize, nK,
                                       thx::as_stream(stream));
}

// The half-map hand-over of Model::compareTwoHemispheres (src/Model.cpp:
// 307-852: MPI_Recv_Large of hemisphere A's and B's maps on the master):
// one point-to-point step on a communicator that spans both hemispheres'
// leads -- `send` (nSend floats) goes to rank peerSend, `recv` (nRecv floats)
// comes from rank peerRecv; either side may be absent (NULL / peer < 0).  Over
// xGMI this is one peer copy; no host staging.
extern "C" int thx_halfmap_sendrecv(void* comm, const float* send, long long nSend, int peerSend,
                                    float* recv, long long nRecv, int peerRecv,
                                    thx_stream_t stream)
{
    THX_CHECK_ARG(comm, "thx_halfmap_sendrecv: null communicator");
    THX_CHECK_ARG(!send || (nSend > 0 && peerSend >= 0), "thx_halfmap_sendrecv: bad send side");
    THX_CHECK_ARG(!recv || (nRecv > 0 && peerRecv >= 0), "thx_halfmap_sendrecv: bad receive side");
    if (!send && !recv) return THX_OK;
    ncclComm_t c = static_cast<ncclComm_t>(comm);
    hipStream_t s = thx::as_stream(stream);
    THX_NCCL(ncclGroupStart());
    ncclResult_t first = ncclSuccess;
    const char* what = "";
    if (send) THX_NCCL_GROUPED(ncclSend(send, (size_t)nSend, ncclFloat32, peerSend, c, s));
    if (recv) THX_NCCL_GROUPED(ncclRecv(recv, (size_t)nRecv, ncclFloat32, peerRecv, c, s));
    return group_end(first, what);
}
