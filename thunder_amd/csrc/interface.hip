// interface.hip -- reference-shaped host adapters over the device C-ABI.
//
// Same argument lists and ownership as gpu/interface/Interface.h (caller owns
// host arrays; the call is stateless: allocate, copy, run, copy back, free),
// so a THUNDER build can forward its Interface.cpp bodies here
// (INTEGRATION.md).  Unlike cuthunder (which round-robins over all visible
// GPUs inside one process, gpu/src/cuthunder.cu:2002-2198), these run on the
// current HIP device: the MI355X layout is one process per GPU.
#include <vector>

#include <cmath>

#include "common.h"

namespace {

// RAII device buffer; errors surface as THX_ERR_NOMEM.
struct DBuf {
    void* p = nullptr;
    hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes > 0 ? bytes : 1); }
    ~DBuf() { if (p) (void)hipFree(p); }
    template <typename T> T* as() const { return static_cast<T*>(p); }
};

#define THX_DALLOC(buf, bytes)                                                 \
    do {                                                                       \
        if ((buf).alloc(bytes) != hipSuccess) {                                \
            thx::set_error("device allocation of %zu bytes failed",           \
                           (size_t)(bytes));                                   \
            return THX_ERR_NOMEM;                                              \
        }                                                                      \
    } while (0)

#define THX_RET(call)                  \
    do {                               \
        int st_ = (call);              \
        if (st_ != THX_OK) return st_; \
    } while (0)

}  // namespace

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
    THX_CHECK_ARG(imgNum >= 0 && nK >= 1 && kIdx >= 0 && kIdx < nK,
                  "thx_ExpectGlobal3D: bad class/image counts");
    if (imgNum == 0) return THX_OK;
    const size_t nPx = (size_t)imgNum * npxl;
    const size_t ws = thx_global_scan_workspace(imgNum, nR, nT, npxl, 1);
    DBuf dRot, dTra, dDat, dCtf, dSig, dWC, dWR, dWT, dPR, dPT, dBase, dWs;
    THX_DALLOC(dRot, sizeof(float) * 2 * (size_t)nR * npxl);
    THX_DALLOC(dTra, sizeof(float) * 2 * (size_t)nT * npxl);
    THX_DALLOC(dDat, sizeof(float) * 2 * nPx);
    THX_DALLOC(dCtf, sizeof(float) * nPx);
    THX_DALLOC(dSig, sizeof(float) * nPx);
    THX_DALLOC(dWC, sizeof(float) * (size_t)imgNum * nK);
    THX_DALLOC(dWR, sizeof(float) * (size_t)imgNum * nK * nR);
    THX_DALLOC(dWT, sizeof(float) * (size_t)imgNum * nK * nT);
    THX_DALLOC(dPR, sizeof(double) * nR);
    THX_DALLOC(dPT, sizeof(double) * nT);
    THX_DALLOC(dBase, sizeof(float) * imgNum);
    THX_DALLOC(dWs, ws);
    THX_HIP(hipMemcpy(dRot.p, rotP, sizeof(float) * 2 * (size_t)nR * npxl, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dTra.p, traP, sizeof(float) * 2 * (size_t)nT * npxl, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dDat.p, datP, sizeof(float) * 2 * nPx, hipMemcpyHostToDevice));
    if (ctfP) THX_HIP(hipMemcpy(dCtf.p, ctfP, sizeof(float) * nPx, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dSig.p, sigRcpP, sizeof(float) * nPx, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dPR.p, pR, sizeof(double) * nR, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dPT.p, pT, sizeof(double) * nT, hipMemcpyHostToDevice));
    if (kIdx > 0) {   // merge into the caller's running accumulation
        THX_HIP(hipMemcpy(dWC.p, wC, sizeof(float) * (size_t)imgNum * nK, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dWR.p, wR, sizeof(float) * (size_t)imgNum * nK * nR, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dWT.p, wT, sizeof(float) * (size_t)imgNum * nK * nT, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dBase.p, baseL, sizeof(float) * imgNum, hipMemcpyHostToDevice));
    }
    THX_RET(thx_global_scan(dRot.as<float>(), nR, dTra.as<float>(), nT, dDat.as<float>(),
                            dCtf.as<float>(), dSig.as<float>(), imgNum, npxl,
                            dPR.as<double>(), dPT.as<double>(), kIdx, nK, dWC.as<float>(),
                            dWR.as<float>(), dWT.as<float>(), dBase.as<float>(), 1, dWs.p,
                            ws, nullptr));
    THX_HIP(hipMemcpy(wC, dWC.p, sizeof(float) * (size_t)imgNum * nK, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(wR, dWR.p, sizeof(float) * (size_t)imgNum * nK * nR, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(wT, dWT.p, sizeof(float) * (size_t)imgNum * nK * nT, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(baseL, dBase.p, sizeof(float) * imgNum, hipMemcpyDeviceToHost));
    return THX_OK;
}

// ctfa / nD (CTF search, both or neither): CTFAttr[imgNum] (7 RFLOAT:
// voltage, defocusU, defocusV, defocusTheta, Cs, amplitudeContrast,
// phaseShift; include/Database.h:302-327) and the samples' defocus factors
// nD[imgNum * mReco]; ctfP is then unused.
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
    THX_CHECK_ARG(imgNum >= 0 && mReco >= 0 && npxl >= 0 && opf > 0, "thx_InsertFT: bad sizes");
    const size_t dimSize = (size_t)(vdim / 2 + 1) * vdim * vdim;
    const size_t nPx = (size_t)imgNum * npxl, nS = (size_t)imgNum * mReco;
    DBuf dF, dT, dO, dC, dDat, dCtf, dOff, dW, dQ, dTr, dIc, dIr, dN, dA, dND;
    THX_DALLOC(dF, sizeof(float) * 2 * dimSize);
    THX_DALLOC(dT, sizeof(float) * dimSize);
    THX_DALLOC(dO, sizeof(double) * 3);
    THX_DALLOC(dC, sizeof(int));
    THX_DALLOC(dDat, sizeof(float) * 2 * nPx);
    THX_DALLOC(dCtf, sizeof(float) * nPx);
    THX_DALLOC(dOff, sizeof(double) * 2 * imgNum);
    THX_DALLOC(dW, sizeof(float) * imgNum);
    THX_DALLOC(dQ, sizeof(double) * 4 * nS);
    THX_DALLOC(dTr, sizeof(double) * 2 * nS);
    THX_DALLOC(dIc, sizeof(int) * npxl);
    THX_DALLOC(dIr, sizeof(int) * npxl);
    THX_DALLOC(dN, sizeof(int) * imgNum);
    if (ctfa) {
        // the thx_ctf attribute rows {pixelSize, voltage, dU, dV, theta, Cs, ampC, ps}
        std::vector<float> a(8 * (size_t)imgNum);
        for (int l = 0; l < imgNum; l++) {
            a[8 * (size_t)l] = pixelSize;
            for (int k = 0; k < 7; k++) a[8 * (size_t)l + 1 + k] = ctfa[7 * (size_t)l + k];
        }
        THX_DALLOC(dA, sizeof(float) * a.size());
        THX_DALLOC(dND, sizeof(double) * nS);
        THX_HIP(hipMemcpy(dA.p, a.data(), sizeof(float) * a.size(), hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dND.p, nD, sizeof(double) * nS, hipMemcpyHostToDevice));
    }
    // the reference seeds GPU0 with the host F/T and accumulates on top
    // (gpu/src/cuthunder.cu:5422-5555)
    THX_HIP(hipMemcpy(dF.p, F3D, sizeof(float) * 2 * dimSize, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dT.p, T3D, sizeof(float) * dimSize, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dO.p, O3D, sizeof(double) * 3, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dC.p, counter, sizeof(int), hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dDat.p, datP, sizeof(float) * 2 * nPx, hipMemcpyHostToDevice));
    if (ctfP) THX_HIP(hipMemcpy(dCtf.p, ctfP, sizeof(float) * nPx, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dOff.p, offS, sizeof(double) * 2 * imgNum, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dW.p, w, sizeof(float) * imgNum, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dQ.p, nR, sizeof(double) * 4 * nS, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dTr.p, nT, sizeof(double) * 2 * nS, hipMemcpyHostToDevice));
    if (nC) THX_HIP(hipMemcpy(dN.p, nC, sizeof(int) * imgNum, hipMemcpyHostToDevice));
    {
        // Reconstructor::insertI passes the padded pixel set (_iCol = iCol * pf,
        // src/Reconstructor.cpp:928-985); the kernels take the unpadded one + pf,
        // as kernel_Translate does with iColPad / opf (gpu/src/Kernel.cu:2088).
        std::vector<int> uc(npxl), ur(npxl);
        for (int i = 0; i < npxl; i++) {
            THX_CHECK_ARG(iCol[i] % opf == 0 && iRow[i] % opf == 0,
                          "thx_InsertFT: iCol/iRow must be the padded (x opf) pixel set");
            uc[i] = iCol[i] / opf;
            ur[i] = iRow[i] / opf;
        }
        THX_HIP(hipMemcpy(dIc.p, uc.data(), sizeof(int) * npxl, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dIr.p, ur.data(), sizeof(int) * npxl, hipMemcpyHostToDevice));
    }
    // the binned deposition where its limits hold (the pixel set's radius
    // and 4x4-patch visiting order from the host copy), else direct atomics
    int rMax = 1;
    std::vector<int> order(16 * (size_t)npxl + 16);
    int nOrd = 0;
    {
        std::vector<int> uc(npxl), ur(npxl);
        for (int i = 0; i < npxl; i++) {
            uc[i] = iCol[i] / opf;
            ur[i] = iRow[i] / opf;
            const int r = (int)std::ceil(std::sqrt((double)uc[i] * uc[i] + (double)ur[i] * ur[i]));
            rMax = r > rMax ? r : rMax;
        }
        THX_RET(thx_pixel_tile_order(uc.data(), ur.data(), npxl, (int)order.size(), order.data(),
                                     &nOrd));
    }
    const size_t binWs = thx_insert3d_binned_workspace(imgNum, mReco, nOrd, opf, rMax);
    const int R = opf * rMax + 2;
    const long nTiles = (long)((R + 15) / 16) * ((2 * R + 15) / 16) * ((2 * R + 15) / 16);
    const bool binned = mReco <= 1024 && R <= vdim / 2 - 1 && nTiles <= 16384;
    THX_CHECK_ARG(!ctfa || binned || imgNum == 0,
                  "thx_InsertFT: the CTF-search insert needs mReco <= 1024 and a tile grid of "
                  "<= 16384 tiles");
    if (binned && imgNum > 0 && ctfa) {
        DBuf dOrd, dWs;
        THX_DALLOC(dOrd, sizeof(int) * nOrd);
        THX_DALLOC(dWs, binWs);
        THX_HIP(hipMemcpy(dOrd.p, order.data(), sizeof(int) * nOrd, hipMemcpyHostToDevice));
        THX_RET(thx_insert3d_binned_d(dF.as<float>(), dT.as<float>(), dO.as<double>(),
                                      dC.as<int>(), vdim, opf, dDat.as<float>(), dA.as<float>(),
                                      dND.as<double>(), dQ.as<double>(), dTr.as<double>(),
                                      dOff.as<double>(), dW.as<float>(),
                                      nC ? dN.as<int>() : nullptr, imgNum, mReco, dIc.as<int>(),
                                      dIr.as<int>(), dOrd.as<int>(), nOrd, npxl, idim, rMax,
                                      dWs.p, binWs, nullptr));
    } else if (binned && imgNum > 0) {
        DBuf dOrd, dWs;
        THX_DALLOC(dOrd, sizeof(int) * nOrd);
        THX_DALLOC(dWs, binWs);
        THX_HIP(hipMemcpy(dOrd.p, order.data(), sizeof(int) * nOrd, hipMemcpyHostToDevice));
        THX_RET(thx_insert3d_binned(dF.as<float>(), dT.as<float>(), dO.as<double>(), dC.as<int>(),
                                    vdim, opf, dDat.as<float>(), dCtf.as<float>(), dQ.as<double>(),
                                    dTr.as<double>(), dOff.as<double>(), dW.as<float>(),
                                    nC ? dN.as<int>() : nullptr, imgNum, mReco, dIc.as<int>(),
                                    dIr.as<int>(), dOrd.as<int>(), nOrd, npxl, idim, rMax, dWs.p,
                                    binWs, nullptr));
    } else {
        for (int l0 = 0; l0 < imgNum; l0 += 65535) {
            const int nb = imgNum - l0 < 65535 ? imgNum - l0 : 65535;
            THX_RET(thx_insert3d(dF.as<float>(), dT.as<float>(), dO.as<double>(), dC.as<int>(),
                                 vdim, opf, dDat.as<float>() + 2 * (size_t)l0 * npxl,
                                 dCtf.as<float>() + (size_t)l0 * npxl,
                                 dQ.as<double>() + 4 * (size_t)l0 * mReco,
                                 dTr.as<double>() + 2 * (size_t)l0 * mReco,
                                 dOff.as<double>() + 2 * (size_t)l0, dW.as<float>() + l0,
                                 nC ? dN.as<int>() + l0 : nullptr, nb, mReco, dIc.as<int>(),
                                 dIr.as<int>(), npxl, idim, nullptr));
        }
    }
    // the hemisphere's all-reduce of the reference call (cuthunder.cu:5903-5993)
    if (comm) {
        THX_RET(thx_halfmap_allreduce(comm, dF.as<float>(), dT.as<float>(), dO.as<double>(),
                                      dC.as<int>(), (long long)dimSize, 1, nullptr));
        THX_HIP(hipDeviceSynchronize());
    }
    THX_HIP(hipMemcpy(F3D, dF.p, sizeof(float) * 2 * dimSize, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(T3D, dT.p, sizeof(float) * dimSize, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(O3D, dO.p, sizeof(double) * 3, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(counter, dC.p, sizeof(int), hipMemcpyDeviceToHost));
    return THX_OK;
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
    const size_t img = (size_t)(vdim / 2 + 1) * vdim, nPx = (size_t)imgNum * npxl;
    const size_t ws = thx_global_scan_workspace(imgNum, nR, nT, npxl, 1);
    DBuf dV, dRot, dTr, dTra, dDat, dCtf, dSig, dWC, dWR, dWT, dPR, dPT, dBase, dWs, dRP, dIc, dIr;
    THX_DALLOC(dV, sizeof(float) * 2 * img * nK);
    THX_DALLOC(dRot, sizeof(double) * 2 * nR);
    THX_DALLOC(dTr, sizeof(double) * 2 * nT);
    THX_DALLOC(dTra, sizeof(float) * 2 * (size_t)nT * npxl);
    THX_DALLOC(dRP, sizeof(float) * 2 * (size_t)nR * npxl);
    THX_DALLOC(dDat, sizeof(float) * 2 * nPx);
    THX_DALLOC(dCtf, sizeof(float) * nPx);
    THX_DALLOC(dSig, sizeof(float) * nPx);
    THX_DALLOC(dWC, sizeof(float) * (size_t)imgNum * nK);
    THX_DALLOC(dWR, sizeof(float) * (size_t)imgNum * nK * nR);
    THX_DALLOC(dWT, sizeof(float) * (size_t)imgNum * nK * nT);
    THX_DALLOC(dPR, sizeof(double) * nR);
    THX_DALLOC(dPT, sizeof(double) * nT);
    THX_DALLOC(dBase, sizeof(float) * imgNum);
    THX_DALLOC(dWs, ws);
    THX_DALLOC(dIc, sizeof(int) * npxl);
    THX_DALLOC(dIr, sizeof(int) * npxl);
    THX_HIP(hipMemcpy(dV.p, vol, sizeof(float) * 2 * img * nK, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dRot.p, rot, sizeof(double) * 2 * nR, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dTr.p, trans, sizeof(double) * 2 * nT, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dDat.p, datP, sizeof(float) * 2 * nPx, hipMemcpyHostToDevice));
    if (ctfP) THX_HIP(hipMemcpy(dCtf.p, ctfP, sizeof(float) * nPx, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dSig.p, sigRcpP, sizeof(float) * nPx, hipMemcpyHostToDevice));
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
                                dCtf.as<float>(), dSig.as<float>(), imgNum, npxl, dPR.as<double>(),
                                dPT.as<double>(), k, nK, dWC.as<float>(), dWR.as<float>(),
                                dWT.as<float>(), dBase.as<float>(), 1, dWs.p, ws, nullptr));
    }
    THX_HIP(hipMemcpy(wC, dWC.p, sizeof(float) * (size_t)imgNum * nK, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(wR, dWR.p, sizeof(float) * (size_t)imgNum * nK * nR, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(wT, dWT.p, sizeof(float) * (size_t)imgNum * nK * nT, hipMemcpyDeviceToHost));
    return THX_OK;
}

extern "C" int thx_InsertI2D(float* F2D, float* T2D, double* O2D, int* counter, const float* datP,
                             const float* ctfP, const float* w, const double* offS, const int* nC,
                             const double* nR, const double* nT, const int* iCol, const int* iRow,
                             int nk, int opf, int npxl, int mReco, int idim, int vdim, int imgNum)
{
    THX_CHECK_ARG(F2D && T2D && O2D && counter && datP && ctfP && w && offS && nC && nR && nT &&
                      iCol && iRow,
                  "thx_InsertI2D: null");
    THX_CHECK_ARG(nk >= 1 && opf > 0 && npxl >= 0 && mReco >= 0 && imgNum >= 0,
                  "thx_InsertI2D: bad sizes");
    const size_t img = (size_t)(vdim / 2 + 1) * vdim, nPx = (size_t)imgNum * npxl;
    const size_t nS = (size_t)imgNum * mReco;
    for (size_t q = 0; q < nS; q++)
        THX_CHECK_ARG(nC[q] >= 0 && nC[q] < nk, "thx_InsertI2D: class index out of range");
    DBuf dF, dT, dO, dC, dDat, dCtf, dW, dOff, dN, dR, dTr, dIc, dIr;
    THX_DALLOC(dF, sizeof(float) * 2 * img * nk);
    THX_DALLOC(dT, sizeof(float) * img * nk);
    THX_DALLOC(dO, sizeof(double) * 2 * nk);
    THX_DALLOC(dC, sizeof(int) * nk);
    THX_DALLOC(dDat, sizeof(float) * 2 * nPx);
    THX_DALLOC(dCtf, sizeof(float) * nPx);
    THX_DALLOC(dW, sizeof(float) * imgNum);
    THX_DALLOC(dOff, sizeof(double) * 2 * imgNum);
    THX_DALLOC(dN, sizeof(int) * nS);
    THX_DALLOC(dR, sizeof(double) * 2 * nS);
    THX_DALLOC(dTr, sizeof(double) * 2 * nS);
    THX_DALLOC(dIc, sizeof(int) * npxl);
    THX_DALLOC(dIr, sizeof(int) * npxl);
    THX_HIP(hipMemcpy(dF.p, F2D, sizeof(float) * 2 * img * nk, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dT.p, T2D, sizeof(float) * img * nk, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dO.p, O2D, sizeof(double) * 2 * nk, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dC.p, counter, sizeof(int) * nk, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dDat.p, datP, sizeof(float) * 2 * nPx, hipMemcpyHostToDevice));
    if (ctfP) THX_HIP(hipMemcpy(dCtf.p, ctfP, sizeof(float) * nPx, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dW.p, w, sizeof(float) * imgNum, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dOff.p, offS, sizeof(double) * 2 * imgNum, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dN.p, nC, sizeof(int) * nS, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dR.p, nR, sizeof(double) * 2 * nS, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(dTr.p, nT, sizeof(double) * 2 * nS, hipMemcpyHostToDevice));
    {
        // the padded pixel set (_iColPad, src/Optimiser.cpp:6823) -> unpadded + opf
        std::vector<int> uc(npxl), ur(npxl);
        for (int i = 0; i < npxl; i++) {
            THX_CHECK_ARG(iCol[i] % opf == 0 && iRow[i] % opf == 0,
                          "thx_InsertI2D: iCol/iRow must be the padded (x opf) pixel set");
            uc[i] = iCol[i] / opf;
            ur[i] = iRow[i] / opf;
        }
        THX_HIP(hipMemcpy(dIc.p, uc.data(), sizeof(int) * npxl, hipMemcpyHostToDevice));
        THX_HIP(hipMemcpy(dIr.p, ur.data(), sizeof(int) * npxl, hipMemcpyHostToDevice));
    }
    for (int l0 = 0; l0 < imgNum; l0 += 65535) {
        const int nb = imgNum - l0 < 65535 ? imgNum - l0 : 65535;
        THX_RET(thx_insert2d(dF.as<float>(), dT.as<float>(), dO.as<double>(), dC.as<int>(), vdim,
                             opf, dDat.as<float>() + 2 * (size_t)l0 * npxl,
                             dCtf.as<float>() + (size_t)l0 * npxl,
                             dR.as<double>() + 2 * (size_t)l0 * mReco,
                             dTr.as<double>() + 2 * (size_t)l0 * mReco, dOff.as<double>() + 2 * l0,
                             dW.as<float>() + l0, dN.as<int>() + (size_t)l0 * mReco, nb, mReco,
                             dIc.as<int>(), dIr.as<int>(), npxl, idim, nullptr));
    }
    THX_HIP(hipMemcpy(F2D, dF.p, sizeof(float) * 2 * img * nk, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(T2D, dT.p, sizeof(float) * img * nk, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(O2D, dO.p, sizeof(double) * 2 * nk, hipMemcpyDeviceToHost));
    THX_HIP(hipMemcpy(counter, dC.p, sizeof(int) * nk, hipMemcpyDeviceToHost));
    return THX_OK;
}
