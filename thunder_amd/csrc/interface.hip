// interface.hip -- reference-shaped host adapters over the device C-ABI.
//
// Same argument lists and ownership as gpu/interface/Interface.h (caller owns
// host arrays; the call is stateless: allocate, copy, run, copy back, free),
// so a THUNDER build can forward its Interface.cpp bodies here
// (INTEGRATION.md).
//
// Devices.  cuthunder deals the image batches of ExpectGlobal3D / 2D and of
// InsertFT / InsertI2D round-robin over every visible GPU of the process
// (gpu/src/cuthunder.cu:2002-2198, 5570-5826, 3265-4033).  The batch adapters
// here do the same over thx_adapter_devices(): every GPU thx_getAviDevice
// reports, or the list in THX_DEVICES ("0,3"), or -- for one process per GPU
// -- the caller's current device alone when THX_DEVICES=current.  Each device
// takes one contiguous block of images in its own host thread; the insert's
// partial half-maps are summed onto the first device by peer copies, then the
// hemisphere's RCCL all-reduce (if a communicator is given) runs there.
// ExpectRotran / ExpectProject run on the current device, as the reference
// runs them on one GPU.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "adapter.h"

using thx::DBuf;
using thx::DeviceGuard;
using thx::on_devices;

namespace {

// the global scan of the batch adapters: bf16x6 (FP32-equivalent products,
// cancellation-guarded), the expectation driver's default
constexpr int kScanAlgo = 4;

template <typename T>
__global__ void k_add(T* __restrict__ dst, const T* __restrict__ src, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        dst[i] += src[i];
}

// dst (on device d0) += src (on device d1): a peer copy into tmp, then an add.
template <typename T>
int add_peer(T* dst, int d0, const T* src, int d1, size_t n, T* tmp)
{
    if (n == 0) return THX_OK;
    THX_HIP(hipSetDevice(d0));
    THX_HIP(hipMemcpyPeer(tmp, d0, src, d1, sizeof(T) * n));
    hipLaunchKernelGGL(k_add<T>, dim3(2048), dim3(256), 0, nullptr, dst, tmp, n);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

// Unpadded pixel set of the Reconstructor's padded one (_iColPad =
// iCol * pf, src/Optimiser.cpp:6823 / src/Reconstructor.cpp:928-985).
int unpad_pixels(const int* iCol, const int* iRow, int npxl, int opf, std::vector<int>& uc,
                 std::vector<int>& ur, int& rMax, const char* who)
{
    uc.resize(npxl);
    ur.resize(npxl);
    rMax = 1;
    for (int i = 0; i < npxl; i++) {
        THX_CHECK_ARG(iCol[i] % opf == 0 && iRow[i] % opf == 0,
                      "%s: iCol/iRow must be the padded (x opf) pixel set", who);
        uc[i] = iCol[i] / opf;
        ur[i] = iRow[i] / opf;
        const int r = (int)std::ceil(std::sqrt((double)uc[i] * uc[i] + (double)ur[i] * ur[i]));
        rMax = r > rMax ? r : rMax;
    }
    return THX_OK;
}

// the thx_ctf attribute rows {pixelSize, voltage, dU, dV, theta, Cs, ampC, ps}
// from CTFAttr (7 RFLOAT: voltage, defocusU, defocusV, defocusTheta, Cs,
// amplitudeContrast, phaseShift; include/Database.h:302-327)
std::vector<float> attr_rows(const float* ctfa, float pixelSize, int l0, int l1)
{
    std::vector<float> a(8 * (size_t)(l1 - l0));
    for (int l = l0; l < l1; l++) {
        a[8 * (size_t)(l - l0)] = pixelSize;
        for (int k = 0; k < 7; k++) a[8 * (size_t)(l - l0) + 1 + k] = ctfa[7 * (size_t)l + k];
    }
    return a;
}

// binned-insert entries per host-adapter call: bounds the workspace a single
// InsertFT reserves (2^24 entries x 24 B = 384 MiB) by inserting in image chunks
constexpr long ADAPTER_BIN_ENTRIES = 1L << 24;

}  // namespace

namespace thx {

// the process's local rank from the launcher's environment (-1: none)
static int local_rank_env()
{
    for (const char* v : {"LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID",
                          "MV2_COMM_WORLD_LOCAL_RANK", "SLURM_LOCALID", "PMI_LOCAL_RANK"}) {
        const char* e = std::getenv(v);
        if (e && *e) return std::atoi(e);
    }
    return -1;
}

// the number of processes the launcher placed on this node (-1: unknown)
static int local_size_env()
{
    for (const char* v : {"LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS",
                          "MV2_COMM_WORLD_LOCAL_SIZE", "SLURM_NTASKS_PER_NODE", "PMI_LOCAL_SIZE"}) {
        const char* e = std::getenv(v);
        if (e && *e) return std::atoi(e);
    }
    return -1;
}

// The devices the batch adapters spread work over and getAviDevice reports
// (see the file comment), from the visible device count, the caller's current
// device, THX_DEVICES and the launcher's local process count / rank:
//   THX_DEVICES unset -> every visible GPU (the reference's getAviDevice), except
//     when the launcher placed at least as many processes on this node as there
//     are GPUs: then one device per process, (local rank % count) -- a
//     one-process-per-GPU launch must not pile every rank onto every GPU, while
//     THUNDER's master + two hemisphere ranks on an 8-GPU node keep all eight;
//   "current" -> the caller's current device; "local" -> (local rank % count);
//   "all" -> every visible GPU; "0,3" -> a list.
int device_policy(int n, int cur, const char* env, int localSize, int localRank,
                  std::vector<int>& devs)
{
    devs.clear();
    THX_CHECK_ARG(n > 0, "no HIP device");
    if (env && std::strcmp(env, "current") == 0) {
        devs.push_back(cur);
        return THX_OK;
    }
    const bool perGpu = localSize > 1 && localSize >= n && localRank >= 0;
    if ((env && std::strcmp(env, "local") == 0) || ((!env || !*env) && perGpu)) {
        devs.push_back(localRank >= 0 ? localRank % n : cur);
        return THX_OK;
    }
    if (env && *env && std::strcmp(env, "all") != 0) {
        std::string s(env);
        size_t i = 0;
        while (i < s.size()) {
            size_t j = s.find(',', i);
            if (j == std::string::npos) j = s.size();
            const int d = std::atoi(s.substr(i, j - i).c_str());
            THX_CHECK_ARG(d >= 0 && d < n, "THX_DEVICES names device %d of %d", d, n);
            devs.push_back(d);
            i = j + 1;
        }
        THX_CHECK_ARG(!devs.empty(), "THX_DEVICES is empty");
        return THX_OK;
    }
    for (int d = 0; d < n; d++) devs.push_back(d);
    return THX_OK;
}

int adapter_devices(std::vector<int>& devs)
{
    int n = 0, cur = 0;
    THX_HIP(hipGetDeviceCount(&n));
    THX_HIP(hipGetDevice(&cur));
    return device_policy(n, cur, std::getenv("THX_DEVICES"), local_size_env(), local_rank_env(),
                         devs);
}

}  // namespace thx

// the policy alone, for host tests (no device calls)
extern "C" int thx_adapter_device_policy(int nVisible, int cur, const char* env, int localSize,
                                         int localRank, int* devs, int cap, int* n)
{
    THX_CHECK_ARG(n && (cap == 0 || devs), "thx_adapter_device_policy: bad arguments");
    std::vector<int> d;
    THX_RET(thx::device_policy(nVisible, cur, env, localSize, localRank, d));
    *n = (int)d.size();
    for (int k = 0; k < (int)d.size() && k < cap; k++) devs[k] = d[k];
    return THX_OK;
}

using thx::adapter_devices;

extern "C" int thx_set_device(int dev)
{
    THX_HIP(hipSetDevice(dev));
    return THX_OK;
}

extern "C" int thx_adapter_devices(int* devs, int cap, int* n)
{
    THX_CHECK_ARG(n && (cap == 0 || devs), "thx_adapter_devices: bad arguments");
    std::vector<int> d;
    THX_RET(adapter_devices(d));
    for (int i = 0; i < (int)d.size() && i < cap; i++) devs[i] = d[i];
    *n = (int)d.size();
    return THX_OK;
}

extern "C" int thx_ExpectRotran(float* traP, const double* trans,
                                const double* rot, double* rotMat,
                                const int* iCol, const int* iRow, int nR, int nT,
                                int idim, int npxl)
{
    THX_CHECK_ARG(traP && trans && rot && rotMat && iCol && iRow && nR >= 0 &&
                      nT >= 0 && npxl >= 0,
                  "thx_ExpectRotran: bad arguments");
    DBuf dT, dR, dM, dIc, dIr, dTr;
    THX_DALLOC(dT, sizeof(double) * 2 * nT);
    THX_DALLOC(dR, sizeof(double) * 4 * nR);
    THX_DALLOC(dM, sizeof(double) * 9 * nR);
    THX_DALLOC(dIc, sizeof(int) * npxl);
    THX_DALLOC(dIr, sizeof(int) * npxl);
    THX_DALLOC(dTr, sizeof(float) * 2 * (size_t)nT * npxl);
    THX_HIP(hipMemcpy(dT.p, trans, sizeof(double) * 2 * nT, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dR.p, rot, sizeof(double) * 4 * nR, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dIc.p, iCol, sizeof(int) * npxl, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dIr.p, iRow, sizeof(int) * npxl, hipMemcpyHostToDevice));
    THX_RET(thx_trans_table(dT.as<double>(), nT, dIc.as<int>(), dIr.as<int>(), npxl,
                            idim, dTr.as<float>(), nullptr));
    THX_RET(thx_rotmat(dR.as<double>(), nR, dM.as<double>(), nullptr));
    THX_HIP(hipMemcpy(traP, dTr.p, sizeof(float) * 2 * (size_t)nT * npxl,
                      hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(rotMat, dM.p, sizeof(double) * 9 * nR, hipMemcpyDeviceToHost));
    return THX_OK;
}

extern "C" int thx_ExpectProject(const float* vol, float* rotP,
                                 const double* rotMat, const int* iCol,
                                 const int* iRow, int nR, int pf, int interp,
                                 int vdim, int npxl)
{
    THX_CHECK_ARG(vol && rotP && rotMat && iCol && iRow, "thx_ExpectProject: null");
    THX_CHECK_ARG(interp == 1, "thx_ExpectProject: only LINEAR_INTERP (1) is supported");
    const size_t dimSize = (size_t)(vdim / 2 + 1) * vdim * vdim;
    DBuf dV, dM, dIc, dIr, dP;
    THX_DALLOC(dV, sizeof(float) * 2 * dimSize);
    THX_DALLOC(dM, sizeof(double) * 9 * nR);
    THX_DALLOC(dIc, sizeof(int) * npxl);
    THX_DALLOC(dIr, sizeof(int) * npxl);
    THX_DALLOC(dP, sizeof(float) * 2 * (size_t)nR * npxl);
    THX_HIP(hipMemcpy(dV.p, vol, sizeof(float) * 2 * dimSize, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dM.p, rotMat, sizeof(double) * 9 * nR, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dIc.p, iCol, sizeof(int) * npxl, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dIr.p, iRow, sizeof(int) * npxl, hipMemcpyHostToDevice));
    for (int r0 = 0; r0 < nR; r0 += 65535) {
        const int nb = nR - r0 < 65535 ? nR - r0 : 65535;
        THX_RET(thx_project3d(dV.as<float>(), vdim, pf, dM.as<double>() + 9 * (size_t)r0,
                              nb, dIc.as<int>(), dIr.as<int>(), npxl,
                              dP.as<float>() + 2 * (size_t)r0 * npxl, nullptr));
    }
    THX_HIP(hipMemcpy(rotP, dP.p, sizeof(float) * 2 * (size_t)nR * npxl,
                      hipMemcpyDeviceToHost));
    return THX_OK;
}

extern "C" int thx_ExpectGlobal3D(const float* rotP, const float* traP,
                                  const float* datP, const float* ctfP,
                                  const float* sigRcpP, float* wC, float* wR,
                                  float* wT, const double* pR, const double* pT,
                                  float* baseL, int kIdx, int nK, int nR, int nT,
                                  int npxl, int imgNum)
{
    THX_CHECK_ARG(rotP && traP && datP && ctfP && sigRcpP && wC && wR && wT && pR &&
                      pT && baseL,
                  "thx_ExpectGlobal3D: null");
    THX_CHECK_ARG(imgNum >= 0 && nK >= 1 && kIdx >= 0 && kIdx < nK && nR > 0 && nT > 0 &&
                      npxl > 0,
                  "thx_ExpectGlobal3D: bad class/image counts");
    if (imgNum == 0) return THX_OK;
    DeviceGuard guard;
    std::vector<int> devs;
    THX_RET(adapter_devices(devs));
    if ((int)devs.size() > imgNum) devs.resize(imgNum);
    return on_devices(devs, imgNum, [&](int, int, int l0, int l1) -> int {
        const int n = l1 - l0;
        if (n <= 0) return THX_OK;
        const size_t nPx = (size_t)n * npxl, o = (size_t)l0 * npxl;
        const size_t ws = thx_global_scan_workspace(n, nR, nT, npxl, kScanAlgo);
        DBuf dRot, dTra, dDat, dCtf, dSig, dWC, dWR, dWT, dPR, dPT, dBase, dWs;
        THX_DALLOC(dRot, sizeof(float) * 2 * (size_t)nR * npxl);
        THX_DALLOC(dTra, sizeof(float) * 2 * (size_t)nT * npxl);
        THX_DALLOC(dDat, sizeof(float) * 2 * nPx);
        THX_DALLOC(dCtf, sizeof(float) * nPx);
        THX_DALLOC(dSig, sizeof(float) * nPx);
        THX_DALLOC(dWC, sizeof(float) * (size_t)n * nK);
        THX_DALLOC(dWR, sizeof(float) * (size_t)n * nK * nR);
        THX_DALLOC(dWT, sizeof(float) * (size_t)n * nK * nT);
        THX_DALLOC(dPR, sizeof(double) * nR);
        THX_DALLOC(dPT, sizeof(double) * nT);
        THX_DALLOC(dBase, sizeof(float) * n);
        THX_DALLOC(dWs, ws);
        THX_HIP(hipMemcpy(dRot.p, rotP, sizeof(float) * 2 * (size_t)nR * npxl, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dTra.p, traP, sizeof(float) * 2 * (size_t)nT * npxl, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dDat.p, datP + 2 * o, sizeof(float) * 2 * nPx, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dCtf.p, ctfP + o, sizeof(float) * nPx, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dSig.p, sigRcpP + o, sizeof(float) * nPx, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dPR.p, pR, sizeof(double) * nR, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dPT.p, pT, sizeof(double) * nT, hipMemcpyHostToDevice));
        if (kIdx > 0) {   // merge into the caller's running accumulation
            THX_HIP(hipMemcpy(dWC.p, wC + (size_t)l0 * nK, sizeof(float) * (size_t)n * nK,
                              hipMemcpyHostToDevice));
            THX_HIP(hipMemcpy(dWR.p, wR + (size_t)l0 * nK * nR, sizeof(float) * (size_t)n * nK * nR,
                              hipMemcpyHostToDevice));
            THX_HIP(hipMemcpy(dWT.p, wT + (size_t)l0 * nK * nT, sizeof(float) * (size_t)n * nK * nT,
                              hipMemcpyHostToDevice));
            THX_HIP(hipMemcpy(dBase.p, baseL + l0, sizeof(float) * n, hipMemcpyHostToDevice));
        }
        THX_RET(thx_global_scan(dRot.as<float>(), nR, dTra.as<float>(), nT, dDat.as<float>(),
                                dCtf.as<float>(), dSig.as<float>(), n, npxl, dPR.as<double>(),
                                dPT.as<double>(), kIdx, nK, dWC.as<float>(), dWR.as<float>(),
                                dWT.as<float>(), dBase.as<float>(), kScanAlgo, dWs.p, ws, nullptr));
        THX_HIP(hipMemcpy(wC + (size_t)l0 * nK, dWC.p, sizeof(float) * (size_t)n * nK,
                          hipMemcpyDeviceToHost));
        THX_HIP(hipMemcpy(wR + (size_t)l0 * nK * nR, dWR.p, sizeof(float) * (size_t)n * nK * nR,
                          hipMemcpyDeviceToHost));
        THX_HIP(hipMemcpy(wT + (size_t)l0 * nK * nT, dWT.p, sizeof(float) * (size_t)n * nK * nT,
                          hipMemcpyDeviceToHost));
        THX_HIP(hipMemcpy(baseL + l0, dBase.p, sizeof(float) * n, hipMemcpyDeviceToHost));
        return THX_OK;
    });
}

namespace {

// Half-map accumulators of one device (F complex, T real, O, counter) for nk
// classes of `img` voxels each.
struct DevMap {
    DBuf F, T, O, C;
};

int alloc_map(DevMap& m, size_t img, int nk, int oDim, bool seed, const float* F, const float* T,
              const double* O, const int* cnt)
{
    THX_DALLOC(m.F, sizeof(float) * 2 * img * nk);
    THX_DALLOC(m.T, sizeof(float) * img * nk);
    THX_DALLOC(m.O, sizeof(double) * oDim * nk);
    THX_DALLOC(m.C, sizeof(int) * nk);
    if (seed) {
        // the reference seeds GPU0 with the host F/T and accumulates on top
        // (gpu/src/cuthunder.cu:5422-5555); the others start at zero
        THX_HIP(hipMemcpy(m.F.p, F, sizeof(float) * 2 * img * nk, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(m.T.p, T, sizeof(float) * img * nk, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(m.O.p, O, sizeof(double) * oDim * nk, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(m.C.p, cnt, sizeof(int) * nk, hipMemcpyHostToDevice));
    } else {
        THX_HIP(hipMemset(m.F.p, 0, sizeof(float) * 2 * img * nk));
        THX_HIP(hipMemset(m.T.p, 0, sizeof(float) * img * nk));
        THX_HIP(hipMemset(m.O.p, 0, sizeof(double) * oDim * nk));
        THX_HIP(hipMemset(m.C.p, 0, sizeof(int) * nk));
    }
    return THX_OK;
}

// Sum the per-device maps onto maps[0], then (comm != NULL) the hemisphere's
// RCCL all-reduce there (cuthunder.cu:5903-5993), then copy back to the host.
int reduce_maps(std::vector<DevMap>& maps, const std::vector<int>& devs, size_t img, int nk,
                int oDim, void* comm, float* F, float* T, double* O, int* cnt)
{
    const int d0 = devs[0];
    THX_HIP(hipSetDevice(d0));
    if (maps.size() > 1) {
        DBuf tmp;
        THX_DALLOC(tmp, sizeof(float) * 2 * img * nk);
        for (size_t k = 1; k < maps.size(); k++) {
            THX_RET(add_peer(maps[0].F.as<float>(), d0, maps[k].F.as<float>(), devs[k], 2 * img * nk,
                             tmp.as<float>()));
            THX_RET(add_peer(maps[0].T.as<float>(), d0, maps[k].T.as<float>(), devs[k], img * nk,
                             tmp.as<float>()));
            THX_RET(add_peer(maps[0].O.as<double>(), d0, maps[k].O.as<double>(), devs[k],
                             (size_t)oDim * nk, reinterpret_cast<double*>(tmp.p)));
            THX_RET(add_peer(maps[0].C.as<int>(), d0, maps[k].C.as<int>(), devs[k], (size_t)nk,
                             reinterpret_cast<int*>(tmp.p)));
            THX_HIP(hipDeviceSynchronize());
        }
    }
    if (comm) {
        // the communicator must live on the device the partial maps were summed
        // onto (several ranks per node: THX_DEVICES unset or "local" gives each
        // its own device)
        int cdev = -1;
        THX_RET(thx::comm_device(comm, &cdev));
        THX_CHECK_ARG(cdev == d0,
                      "hemisphere communicator on device %d, adapter maps on device %d "
                      "(one device per rank: THX_DEVICES=local)", cdev, d0);
        THX_RET(thx::halfmap_allreduce_impl(comm, maps[0].F.as<float>(), maps[0].T.as<float>(),
                                            maps[0].O.as<double>(), oDim, maps[0].C.as<int>(),
                                            (long long)img, nk, nullptr));
        THX_HIP(hipDeviceSynchronize());
    }
    THX_HIP(hipMemcpy(F, maps[0].F.p, sizeof(float) * 2 * img * nk, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(T, maps[0].T.p, sizeof(float) * img * nk, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(O, maps[0].O.p, sizeof(double) * oDim * nk, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(cnt, maps[0].C.p, sizeof(int) * nk, hipMemcpyDeviceToHost));
    return THX_OK;
}

}  // namespace

// ctfa / nD (CTF search, both or neither): CTFAttr[imgNum] (7 RFLOAT each)
// and the samples' defocus factors nD[imgNum * mReco]; ctfP is then unused.
static int insert_ft(float* F3D, float* T3D, double* O3D, int* counter, const float* datP,
                     const float* ctfP, const double* offS, const float* w, const double* nR,
                     const double* nT, const int* nC, const int* iCol, const int* iRow, int opf,
                     int npxl, int mReco, int idim, int vdim, int imgNum, void* comm,
                     const float* ctfa = nullptr, const double* nD = nullptr,
                     float pixelSize = 0.f)
{
    THX_CHECK_ARG(F3D && T3D && O3D && counter && datP && (ctfP || ctfa) && offS && w && nR &&
                      nT && iCol && iRow && !ctfa == !nD,
                  "thx_InsertFT: null");
    THX_CHECK_ARG(!ctfa || pixelSize > 0.f, "thx_InsertFT: CTF search needs the pixel size");
    THX_CHECK_ARG(imgNum >= 0 && mReco >= 0 && npxl >= 0 && opf > 0 && vdim > 0 && vdim % 2 == 0,
                  "thx_InsertFT: bad sizes");
    const size_t dimSize = (size_t)(vdim / 2 + 1) * vdim * vdim;
    std::vector<int> uc, ur;
    int rMax = 1;
    THX_RET(unpad_pixels(iCol, iRow, npxl, opf, uc, ur, rMax, "thx_InsertFT"));
    // the binned deposition where its limits hold (4x4-patch visiting order
    // from the host copy), else direct atomics
    std::vector<int> order(16 * (size_t)npxl + 16);
    int nOrd = 0;
    if (npxl > 0)
        THX_RET(thx_pixel_tile_order(uc.data(), ur.data(), npxl, (int)order.size(), order.data(),
                                     &nOrd));
    const int R = opf * rMax + 2;
    const long nTiles = (long)((R + 15) / 16) * ((2 * R + 15) / 16) * ((2 * R + 15) / 16);
    const bool binned = mReco <= 1024 && R <= vdim / 2 - 1 && nTiles <= 16384 && npxl > 0;
    THX_CHECK_ARG(!ctfa || binned || imgNum == 0 || npxl == 0,
                  "thx_InsertFT: the CTF-search insert needs mReco <= 1024 and a tile grid of "
                  "<= 16384 tiles");
    DeviceGuard guard;
    std::vector<int> devs;
    THX_RET(adapter_devices(devs));
    if (imgNum < (int)devs.size()) devs.resize(imgNum > 0 ? imgNum : 1);
    std::vector<DevMap> maps(devs.size());
    THX_RET(on_devices(devs, imgNum, [&](int k, int, int l0, int l1) -> int {
        DevMap& m = maps[k];
        THX_RET(alloc_map(m, dimSize, 1, 3, k == 0, F3D, T3D, O3D, counter));
        const int n = l1 - l0;
        if (n <= 0 || mReco == 0 || npxl == 0) return THX_OK;
        const size_t nPx = (size_t)n * npxl, nS = (size_t)n * mReco;
        DBuf dDat, dCtf, dOff, dW, dQ, dTr, dIc, dIr, dN, dA, dND, dOrd;
        THX_DALLOC(dDat, sizeof(float) * 2 * nPx);
        THX_DALLOC(dCtf, sizeof(float) * (ctfa ? 1 : nPx));
        THX_DALLOC(dOff, sizeof(double) * 2 * n);
        THX_DALLOC(dW, sizeof(float) * n);
        THX_DALLOC(dQ, sizeof(double) * 4 * nS);
        THX_DALLOC(dTr, sizeof(double) * 2 * nS);
        THX_DALLOC(dIc, sizeof(int) * npxl);
        THX_DALLOC(dIr, sizeof(int) * npxl);
        THX_DALLOC(dN, sizeof(int) * n);
        THX_DALLOC(dOrd, sizeof(int) * (nOrd > 0 ? nOrd : 1));
        const size_t o = (size_t)l0 * npxl;
        THX_HIP(hipMemcpy(dDat.p, datP + 2 * o, sizeof(float) * 2 * nPx, hipMemcpyHostToDevice));
        if (!ctfa) THX_HIP(hipMemcpy(dCtf.p, ctfP + o, sizeof(float) * nPx, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dOff.p, offS + 2 * (size_t)l0, sizeof(double) * 2 * n, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dW.p, w + l0, sizeof(float) * n, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dQ.p, nR + 4 * (size_t)l0 * mReco, sizeof(double) * 4 * nS,
                          hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dTr.p, nT + 2 * (size_t)l0 * mReco, sizeof(double) * 2 * nS,
                          hipMemcpyHostToDevice));
        if (nC) THX_HIP(hipMemcpy(dN.p, nC + l0, sizeof(int) * n, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dIc.p, uc.data(), sizeof(int) * npxl, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dIr.p, ur.data(), sizeof(int) * npxl, hipMemcpyHostToDevice));
        if (nOrd > 0)
            THX_HIP(hipMemcpy(dOrd.p, order.data(), sizeof(int) * nOrd, hipMemcpyHostToDevice));
        if (ctfa) {
            const std::vector<float> a = attr_rows(ctfa, pixelSize, l0, l1);
            THX_DALLOC(dA, sizeof(float) * a.size());
            THX_DALLOC(dND, sizeof(double) * nS);
            THX_HIP(hipMemcpy(dA.p, a.data(), sizeof(float) * a.size(), hipMemcpyHostToDevice));
            THX_HIP(hipMemcpy(dND.p, nD + (size_t)l0 * mReco, sizeof(double) * nS,
                              hipMemcpyHostToDevice));
        }
        float *F = m.F.as<float>(), *T = m.T.as<float>();
        double* O = m.O.as<double>();
        int* C = m.C.as<int>();
        if (binned) {
            // image chunks of <= ADAPTER_BIN_ENTRIES binned entries
            const long perImg = (long)mReco * nOrd;
            const int chunk = (int)std::max(1L, std::min((long)n, ADAPTER_BIN_ENTRIES / perImg));
            const size_t binWs = thx_insert3d_binned_workspace(chunk, mReco, nOrd, opf, rMax);
            DBuf dWs;
            THX_DALLOC(dWs, binWs);
            for (int c0 = 0; c0 < n; c0 += chunk) {
                const int nb = std::min(chunk, n - c0);
                const size_t cp = (size_t)c0 * npxl, cs = (size_t)c0 * mReco;
                if (ctfa)
                    THX_RET(thx_insert3d_binned_d(
                        F, T, O, C, vdim, opf, dDat.as<float>() + 2 * cp, dA.as<float>() + 8 * c0,
                        dND.as<double>() + cs, dQ.as<double>() + 4 * cs, dTr.as<double>() + 2 * cs,
                        dOff.as<double>() + 2 * c0, dW.as<float>() + c0,
                        nC ? dN.as<int>() + c0 : nullptr, nb, mReco, dIc.as<int>(), dIr.as<int>(),
                        dOrd.as<int>(), nOrd, npxl, idim, rMax, dWs.p, binWs, nullptr));
                else
                    THX_RET(thx_insert3d_binned(
                        F, T, O, C, vdim, opf, dDat.as<float>() + 2 * cp, dCtf.as<float>() + cp,
                        dQ.as<double>() + 4 * cs, dTr.as<double>() + 2 * cs,
                        dOff.as<double>() + 2 * c0, dW.as<float>() + c0,
                        nC ? dN.as<int>() + c0 : nullptr, nb, mReco, dIc.as<int>(), dIr.as<int>(),
                        dOrd.as<int>(), nOrd, npxl, idim, rMax, dWs.p, binWs, nullptr));
            }
        } else {
            for (int c0 = 0; c0 < n; c0 += 65535) {
                const int nb = n - c0 < 65535 ? n - c0 : 65535;
                THX_RET(thx_insert3d(F, T, O, C, vdim, opf, dDat.as<float>() + 2 * (size_t)c0 * npxl,
                                     dCtf.as<float>() + (size_t)c0 * npxl,
                                     dQ.as<double>() + 4 * (size_t)c0 * mReco,
                                     dTr.as<double>() + 2 * (size_t)c0 * mReco,
                                     dOff.as<double>() + 2 * (size_t)c0, dW.as<float>() + c0,
                                     nC ? dN.as<int>() + c0 : nullptr, nb, mReco, dIc.as<int>(),
                                     dIr.as<int>(), npxl, idim, nullptr));
            }
        }
        THX_HIP(hipDeviceSynchronize());
        return THX_OK;
    }));
    return reduce_maps(maps, devs, dimSize, 1, 3, comm, F3D, T3D, O3D, counter);
}

extern "C" int thx_InsertFT(float* F3D, float* T3D, double* O3D, int* counter,
                            const float* datP, const float* ctfP,
                            const double* offS, const float* w, const double* nR,
                            const double* nT, const int* iCol, const int* iRow,
                            int opf, int npxl, int mReco, int idim, int vdim,
                            int imgNum)
{
    return insert_ft(F3D, T3D, O3D, counter, datP, ctfP, offS, w, nR, nT, nullptr, iCol, iRow,
                     opf, npxl, mReco, idim, vdim, imgNum, nullptr);
}

extern "C" int thx_InsertFTCS(float* F3D, float* T3D, double* O3D, int* counter,
                              const float* datP, const float* ctfaData, const double* offS,
                              const float* w, const double* nR, const double* nT,
                              const double* nD, const int* nC, const int* iCol, const int* iRow,
                              float pixelSize, int opf, int npxl, int mReco, int idim, int vdim,
                              int imgNum, void* comm)
{
    THX_CHECK_ARG(ctfaData && nD, "thx_InsertFTCS: ctfaData and nD are required");
    return insert_ft(F3D, T3D, O3D, counter, datP, nullptr, offS, w, nR, nT, nC, iCol, iRow, opf,
                     npxl, mReco, idim, vdim, imgNum, comm, ctfaData, nD, pixelSize);
}

extern "C" int thx_InsertFTC(float* F3D, float* T3D, double* O3D, int* counter,
                             const float* datP, const float* ctfP, const double* offS,
                             const float* w, const double* nR, const double* nT, const int* nC,
                             const int* iCol, const int* iRow, int opf, int npxl, int mReco,
                             int idim, int vdim, int imgNum)
{
    THX_CHECK_ARG(nC, "thx_InsertFTC: null nC");
    return insert_ft(F3D, T3D, O3D, counter, datP, ctfP, offS, w, nR, nT, nC, iCol, iRow, opf,
                     npxl, mReco, idim, vdim, imgNum, nullptr);
}

extern "C" int thx_InsertFTComm(float* F3D, float* T3D, double* O3D, int* counter,
                                const float* datP, const float* ctfP, const double* offS,
                                const float* w, const double* nR, const double* nT,
                                const int* nC, const int* iCol, const int* iRow, int opf,
                                int npxl, int mReco, int idim, int vdim, int imgNum, void* comm)
{
    return insert_ft(F3D, T3D, O3D, counter, datP, ctfP, offS, w, nR, nT, nC, iCol, iRow, opf,
                     npxl, mReco, idim, vdim, imgNum, comm);
}

// ---- 2D (MODE_2D) host adapters
extern "C" int thx_ExpectGlobal2D(const float* vol, const float* datP, const float* ctfP,
                                  const float* sigRcpP, const double* trans, float* wC, float* wR,
                                  float* wT, const double* pR, const double* pT, const double* rot,
                                  const int* iCol, const int* iRow, int nK, int nR, int nT, int pf,
                                  int interp, int idim, int vdim, int npxl, int imgNum)
{
    THX_CHECK_ARG(vol && datP && ctfP && sigRcpP && trans && wC && wR && wT && pR && pT && rot &&
                      iCol && iRow,
                  "thx_ExpectGlobal2D: null");
    THX_CHECK_ARG(interp == 1, "thx_ExpectGlobal2D: only LINEAR_INTERP (1) is supported");
    THX_CHECK_ARG(nK >= 1 && nR > 0 && nT > 0 && npxl > 0 && imgNum >= 0 && vdim == pf * idim,
                  "thx_ExpectGlobal2D: bad sizes");
    if (imgNum == 0) return THX_OK;
    const size_t img = (size_t)(vdim / 2 + 1) * vdim;
    DeviceGuard guard;
    std::vector<int> devs;
    THX_RET(adapter_devices(devs));
    if ((int)devs.size() > imgNum) devs.resize(imgNum);
    return on_devices(devs, imgNum, [&](int, int, int l0, int l1) -> int {
        const int n = l1 - l0;
        if (n <= 0) return THX_OK;
        const size_t nPx = (size_t)n * npxl, o = (size_t)l0 * npxl;
        const size_t ws = thx_global_scan_workspace(n, nR, nT, npxl, kScanAlgo);
        DBuf dV, dRot, dTr, dTra, dDat, dCtf, dSig, dWC, dWR, dWT, dPR, dPT, dBase, dWs, dRP, dIc, dIr;
        THX_DALLOC(dV, sizeof(float) * 2 * img * nK);
        THX_DALLOC(dRot, sizeof(double) * 2 * nR);
        THX_DALLOC(dTr, sizeof(double) * 2 * nT);
        THX_DALLOC(dTra, sizeof(float) * 2 * (size_t)nT * npxl);
        THX_DALLOC(dRP, sizeof(float) * 2 * (size_t)nR * npxl);
        THX_DALLOC(dDat, sizeof(float) * 2 * nPx);
        THX_DALLOC(dCtf, sizeof(float) * nPx);
        THX_DALLOC(dSig, sizeof(float) * nPx);
        THX_DALLOC(dWC, sizeof(float) * (size_t)n * nK);
        THX_DALLOC(dWR, sizeof(float) * (size_t)n * nK * nR);
        THX_DALLOC(dWT, sizeof(float) * (size_t)n * nK * nT);
        THX_DALLOC(dPR, sizeof(double) * nR);
        THX_DALLOC(dPT, sizeof(double) * nT);
        THX_DALLOC(dBase, sizeof(float) * n);
        THX_DALLOC(dWs, ws);
        THX_DALLOC(dIc, sizeof(int) * npxl);
        THX_DALLOC(dIr, sizeof(int) * npxl);
        THX_HIP(hipMemcpy(dV.p, vol, sizeof(float) * 2 * img * nK, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dRot.p, rot, sizeof(double) * 2 * nR, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dTr.p, trans, sizeof(double) * 2 * nT, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dDat.p, datP + 2 * o, sizeof(float) * 2 * nPx, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dCtf.p, ctfP + o, sizeof(float) * nPx, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dSig.p, sigRcpP + o, sizeof(float) * nPx, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dPR.p, pR, sizeof(double) * nR, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dPT.p, pT, sizeof(double) * nT, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dIc.p, iCol, sizeof(int) * npxl, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dIr.p, iRow, sizeof(int) * npxl, hipMemcpyHostToDevice));
        THX_RET(thx_trans_table(dTr.as<double>(), nT, dIc.as<int>(), dIr.as<int>(), npxl, idim,
                                dTra.as<float>(), nullptr));
        for (int k = 0; k < nK; k++) {
            // every class against the shared samples, one running baseline (expectGlobal2D)
            THX_RET(thx_project2d(dV.as<float>() + 2 * img * k, vdim, pf, dRot.as<double>(), nR,
                                  dIc.as<int>(), dIr.as<int>(), npxl, dRP.as<float>(), nullptr));
            THX_RET(thx_global_scan(dRP.as<float>(), nR, dTra.as<float>(), nT, dDat.as<float>(),
                                    dCtf.as<float>(), dSig.as<float>(), n, npxl, dPR.as<double>(),
                                    dPT.as<double>(), k, nK, dWC.as<float>(), dWR.as<float>(),
                                    dWT.as<float>(), dBase.as<float>(), kScanAlgo, dWs.p, ws, nullptr));
        }
        THX_HIP(hipMemcpy(wC + (size_t)l0 * nK, dWC.p, sizeof(float) * (size_t)n * nK,
                          hipMemcpyDeviceToHost));
        THX_HIP(hipMemcpy(wR + (size_t)l0 * nK * nR, dWR.p, sizeof(float) * (size_t)n * nK * nR,
                          hipMemcpyDeviceToHost));
        THX_HIP(hipMemcpy(wT + (size_t)l0 * nK * nT, dWT.p, sizeof(float) * (size_t)n * nK * nT,
                          hipMemcpyDeviceToHost));
        return THX_OK;
    });
}

// gpu/interface/Interface.h:239-265 InsertI2D, argument for argument; the
// (hemi, slav) MPI pair becomes `comm`, the hemisphere's RCCL communicator
// (NULL: no reduction); sigRcpP is unused, as in the reference build
// (OPTIMISER_RECONSTRUCT_SIGMA_REGULARISE is off, include/Config.h).
extern "C" int thx_InsertI2D(float* F2D, float* T2D, double* O2D, int* counter, void* comm,
                             const float* datP, const float* ctfP, const float* sigRcpP,
                             const float* w, const double* offS, const int* nC, const double* nR,
                             const double* nT, const double* nD, const float* ctfaData,
                             const int* iCol, const int* iRow, float pixelSize, int cSearch,
                             int nk, int opf, int npxl, int mReco, int idim, int vdim, int imgNum)
{
    (void)sigRcpP;
    THX_CHECK_ARG(F2D && T2D && O2D && counter && datP && w && offS && nC && nR && nT && iCol &&
                      iRow,
                  "thx_InsertI2D: null");
    THX_CHECK_ARG(cSearch ? (ctfaData && nD && pixelSize > 0.f) : (ctfP != nullptr),
                  "thx_InsertI2D: cSearch needs ctfaData, nD and the pixel size; else ctfP");
    THX_CHECK_ARG(nk >= 1 && opf > 0 && npxl >= 0 && mReco >= 0 && imgNum >= 0 && vdim > 0 &&
                      vdim % 2 == 0,
                  "thx_InsertI2D: bad sizes");
    const size_t img = (size_t)(vdim / 2 + 1) * vdim;
    const size_t nSAll = (size_t)imgNum * mReco;
    for (size_t q = 0; q < nSAll; q++)
        THX_CHECK_ARG(nC[q] >= 0 && nC[q] < nk, "thx_InsertI2D: class index out of range");
    std::vector<int> uc, ur;
    int rMax = 1;
    THX_RET(unpad_pixels(iCol, iRow, npxl, opf, uc, ur, rMax, "thx_InsertI2D"));
    DeviceGuard guard;
    std::vector<int> devs;
    THX_RET(adapter_devices(devs));
    if (imgNum < (int)devs.size()) devs.resize(imgNum > 0 ? imgNum : 1);
    std::vector<DevMap> maps(devs.size());
    THX_RET(on_devices(devs, imgNum, [&](int k, int, int l0, int l1) -> int {
        DevMap& m = maps[k];
        THX_RET(alloc_map(m, img, nk, 2, k == 0, F2D, T2D, O2D, counter));
        const int n = l1 - l0;
        if (n <= 0 || mReco == 0 || npxl == 0) return THX_OK;
        const size_t nPx = (size_t)n * npxl, nS = (size_t)n * mReco, o = (size_t)l0 * npxl;
        DBuf dDat, dCtf, dW, dOff, dN, dR, dTr, dIc, dIr, dA, dND;
        THX_DALLOC(dDat, sizeof(float) * 2 * nPx);
        THX_DALLOC(dCtf, sizeof(float) * (cSearch ? 1 : nPx));
        THX_DALLOC(dW, sizeof(float) * n);
        THX_DALLOC(dOff, sizeof(double) * 2 * n);
        THX_DALLOC(dN, sizeof(int) * nS);
        THX_DALLOC(dR, sizeof(double) * 2 * nS);
        THX_DALLOC(dTr, sizeof(double) * 2 * nS);
        THX_DALLOC(dIc, sizeof(int) * npxl);
        THX_DALLOC(dIr, sizeof(int) * npxl);
        THX_HIP(hipMemcpy(dDat.p, datP + 2 * o, sizeof(float) * 2 * nPx, hipMemcpyHostToDevice));
        if (!cSearch) THX_HIP(hipMemcpy(dCtf.p, ctfP + o, sizeof(float) * nPx, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dW.p, w + l0, sizeof(float) * n, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dOff.p, offS + 2 * (size_t)l0, sizeof(double) * 2 * n, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dN.p, nC + (size_t)l0 * mReco, sizeof(int) * nS, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dR.p, nR + 2 * (size_t)l0 * mReco, sizeof(double) * 2 * nS,
                          hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dTr.p, nT + 2 * (size_t)l0 * mReco, sizeof(double) * 2 * nS,
                          hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dIc.p, uc.data(), sizeof(int) * npxl, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dIr.p, ur.data(), sizeof(int) * npxl, hipMemcpyHostToDevice));
        if (cSearch) {
            const std::vector<float> a = attr_rows(ctfaData, pixelSize, l0, l1);
            THX_DALLOC(dA, sizeof(float) * a.size());
            THX_DALLOC(dND, sizeof(double) * nS);
            THX_HIP(hipMemcpy(dA.p, a.data(), sizeof(float) * a.size(), hipMemcpyHostToDevice));
            THX_HIP(hipMemcpy(dND.p, nD + (size_t)l0 * mReco, sizeof(double) * nS,
                              hipMemcpyHostToDevice));
        }
        for (int c0 = 0; c0 < n; c0 += 65535) {
            const int nb = n - c0 < 65535 ? n - c0 : 65535;
            const size_t cp = (size_t)c0 * npxl, cs = (size_t)c0 * mReco;
            if (cSearch)
                THX_RET(thx_insert2d_d(m.F.as<float>(), m.T.as<float>(), m.O.as<double>(),
                                       m.C.as<int>(), vdim, opf, dDat.as<float>() + 2 * cp,
                                       dA.as<float>() + 8 * (size_t)c0, dND.as<double>() + cs,
                                       dR.as<double>() + 2 * cs, dTr.as<double>() + 2 * cs,
                                       dOff.as<double>() + 2 * c0, dW.as<float>() + c0,
                                       dN.as<int>() + cs, nb, mReco, dIc.as<int>(), dIr.as<int>(),
                                       npxl, idim, nullptr));
            else
                THX_RET(thx_insert2d(m.F.as<float>(), m.T.as<float>(), m.O.as<double>(),
                                     m.C.as<int>(), vdim, opf, dDat.as<float>() + 2 * cp,
                                     dCtf.as<float>() + cp, dR.as<double>() + 2 * cs,
                                     dTr.as<double>() + 2 * cs, dOff.as<double>() + 2 * c0,
                                     dW.as<float>() + c0, dN.as<int>() + cs, nb, mReco,
                                     dIc.as<int>(), dIr.as<int>(), npxl, idim, nullptr));
        }
        THX_HIP(hipDeviceSynchronize());
        return THX_OK;
    }));
    return reduce_maps(maps, devs, img, nk, 2, comm, F2D, T2D, O2D, counter);
}
