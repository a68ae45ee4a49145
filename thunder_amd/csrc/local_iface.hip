// local_iface.hip -- the reference's per-image local-search plugin surface
// (gpu/interface/Interface.h:16-164: getAviDevice, ExpectPreidx, ExpectPrefre,
// ExpectLocalIn, ExpectLocalV3D, ExpectLocalP, ExpectLocalHostA / HostF,
// ExpectLocalRTD, ExpectLocalPreI3D, ExpectLocalM, ExpectLocalFin,
// ExpectFreeIdx) over the device C-ABI, so the OpenMP image loop of
// Optimiser::expectationG (src/Optimiser.cpp:2160-2750) can run unchanged on
// MI355X with each Interface.cpp body a one-line forward.
//
// The reference's stateful handles become opaque thx handles:
//   ManagedArrayTexture (gpu/include/ManagedArrayTexture.h) -> thx_tex: the
//     half-complex projectee resident in device memory (no texture object:
//     the fused kernel gathers from LDS patch boxes or plain global loads);
//   ManagedCalPoint (gpu/include/ManagedCalPoint.h) -> thx_calpoint: one
//     image's sample set, priors, marginals and the local-phase workspace on a
//     HIP stream of its own.
// ExpectLocalPreI3D (projection tables, cuthunder.cu:2834) only binds the
// volume, pixel set and geometry to the calpoint; ExpectLocalM runs the fused
// projection + likelihood + marginals (thx_local_phase for one image) and
// copies wC / wR / wT / wD back, synchronising the calpoint's stream as the
// reference does (cuthunder.cu:3140).  CTF search (searchType 2 / cSearch):
// ExpectLocalIn also allocates the per-pixel defocus slots, ExpectLocalP
// fills them, ExpectLocalRTD uploads the defocus factors (dpara) and their
// priors (oldD), ExpectLocalPreI3D computes the calpoint's CTF per defocus
// sample (kernel_CalCTFL, cuthunder.cu:2796-2810) and ExpectLocalM runs the
// (r, t, d) phase (thx_local_phase_d) and returns wD.
// This per-image path exists for drop-in compatibility; thx_expectation runs
// the same phases for the whole batch on device.
#include <vector>

#include "common.h"

namespace {

struct Tex {
    int vdim = 0, gpu = 0, mode = 1;   // mode 1: 3D projectee, 0: one 2D class image
    float* vol = nullptr;   // dimSize Complex
};

struct CalPoint {
    int gpu = 0, mR = 0, mT = 0, npxl = 0, mD = 1, mode = 1;
    double* rot2 = nullptr;                               // 2D: (cos, sin) per rotation
    bool cs = false;                                      // SEARCH_TYPE_CTF
    double *dP = nullptr, *pD = nullptr;                  // defocus factors, priors
    float *ctfD = nullptr, *wD = nullptr;                 // CTF per sample, marginal
    hipStream_t stream = nullptr;
    double *quat = nullptr, *trans = nullptr, *pR = nullptr, *pT = nullptr, *pC = nullptr;
    float *wC = nullptr, *wR = nullptr, *wT = nullptr, *base = nullptr;
    int* order = nullptr;     // tile order of the bound pixel set
    int nOrd = 0;
    const int* boundCol = nullptr;
    void* ws = nullptr;
    size_t wsBytes = 0;
    // bound by PreI3D
    const Tex* tex = nullptr;
    const int *iCol = nullptr, *iRow = nullptr;
    int pf = 0, idim = 0, vdim = 0;
};

#define THX_DEV_SET(g) THX_HIP(hipSetDevice(g))

template <typename T>
int dalloc(T** p, size_t n)
{
    THX_HIP(hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * (n > 0 ? n : 1)));
    return THX_OK;
}

__global__ void k_rot2_from_quat(const double* __restrict__ quat, int n, double* __restrict__ rot2)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    rot2[2 * k] = quat[4 * k];
    rot2[2 * k + 1] = quat[4 * k + 1];
}

// kernel_CalCTFL for one calpoint: ctfD[d][i] from the image's per-pixel
// defocus, the frequencies and the calpoint's defocus factors
__global__ void __launch_bounds__(256) k_calpoint_ctf(const float* __restrict__ dfo,
                                                      const float* __restrict__ freq,
                                                      const double* __restrict__ dP, float ps,
                                                      float conT, float k1, float k2, int npxl,
                                                      float* __restrict__ ctfD)
{
    const double d = dP[blockIdx.y];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < npxl; i += gridDim.x * blockDim.x)
        ctfD[(size_t)blockIdx.y * npxl + i] = ctf_search_at(k1, dfo[i], d, freq[i], k2, ps, conT);
}

}  // namespace

extern "C" int thx_getAviDevice(int* gpus, int cap, int* n)
{
    THX_CHECK_ARG(n && (cap == 0 || gpus), "thx_getAviDevice: bad arguments");
    // the adapter devices (every GPU, or THX_DEVICES: one per process with "local")
    std::vector<int> d;
    const int st = thx::adapter_devices(d);
    if (st != THX_OK) return st;
    for (int i = 0; i < (int)d.size() && i < cap; i++) gpus[i] = d[i];
    *n = (int)d.size();
    return THX_OK;
}

extern "C" int thx_ExpectPreidx(int gpuIdx, int** deviCol, int** deviRow, const int* iCol,
                                const int* iRow, int npxl)
{
    THX_CHECK_ARG(deviCol && deviRow && iCol && iRow && npxl > 0, "thx_ExpectPreidx: bad arguments");
    THX_DEV_SET(gpuIdx);
    THX_RET(dalloc(deviCol, npxl));
    THX_RET(dalloc(deviRow, npxl));
    THX_HIP(hipMemcpy(*deviCol, iCol, sizeof(int) * npxl, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(*deviRow, iRow, sizeof(int) * npxl, hipMemcpyHostToDevice));
    return THX_OK;
}

extern "C" int thx_ExpectPrefre(int gpuIdx, float** devfreQ, const float* freQ, int npxl)
{
    THX_CHECK_ARG(devfreQ && npxl > 0, "thx_ExpectPrefre: bad arguments");
    THX_DEV_SET(gpuIdx);
    THX_RET(dalloc(devfreQ, npxl));
    if (freQ) THX_HIP(hipMemcpy(*devfreQ, freQ, sizeof(float) * npxl, hipMemcpyHostToDevice));
    return THX_OK;
}

extern "C" int thx_ExpectFreeIdx(int gpuIdx, int** deviCol, int** deviRow)
{
    THX_DEV_SET(gpuIdx);
    if (deviCol && *deviCol) { THX_HIP(hipFree(*deviCol)); *deviCol = nullptr; }
    if (deviRow && *deviRow) { THX_HIP(hipFree(*deviRow)); *deviRow = nullptr; }
    return THX_OK;
}

extern "C" int thx_ExpectLocalIn(int gpuIdx, float** devdatP, float** devctfP, float** devdefO,
                                 float** devsigP, int nPxl, int cpyNumL, int searchType)
{
    THX_CHECK_ARG(devdatP && devctfP && devsigP && nPxl > 0 && cpyNumL > 0,
                  "thx_ExpectLocalIn: bad arguments");
    THX_CHECK_ARG(searchType != 2 || devdefO, "thx_ExpectLocalIn: CTF search needs devdefO");
    THX_DEV_SET(gpuIdx);
    const size_t n = (size_t)nPxl * cpyNumL;
    THX_RET(dalloc(devdatP, 2 * n));
    THX_RET(dalloc(devctfP, n));
    THX_RET(dalloc(devsigP, n));
    if (searchType == 2) THX_RET(dalloc(devdefO, n));
    else if (devdefO) *devdefO = nullptr;
    return THX_OK;
}

extern "C" int thx_ExpectLocalP(int gpuIdx, float* devdatP, float* devctfP, float* devdefO,
                                float* devsigP, const float* datP, const float* ctfP,
                                const float* defO, const float* sigP, int threadId, int imgId,
                                int npxl, int cSearch)
{
    THX_CHECK_ARG(devdatP && devctfP && devsigP && datP && (ctfP || cSearch) && sigP &&
                      threadId >= 0 && imgId >= 0 && npxl > 0 &&
                      (!cSearch || (devdefO && defO)),
                  "thx_ExpectLocalP: bad arguments");
    THX_DEV_SET(gpuIdx);
    const size_t d = (size_t)threadId * npxl, s = (size_t)imgId * npxl;
    THX_HIP(hipMemcpy(devdatP + 2 * d, datP + 2 * s, sizeof(float) * 2 * npxl, hipMemcpyHostToDevice));
    if (ctfP)
        THX_HIP(hipMemcpy(devctfP + d, ctfP + s, sizeof(float) * npxl, hipMemcpyHostToDevice));
    if (cSearch)
        THX_HIP(hipMemcpy(devdefO + d, defO + s, sizeof(float) * npxl, hipMemcpyHostToDevice));
    THX_HIP(hipMemcpy(devsigP + d, sigP + s, sizeof(float) * npxl, hipMemcpyHostToDevice));
    return THX_OK;
}

extern "C" int thx_ExpectLocalFin(int gpuIdx, float** devdatP, float** devctfP, float** devdefO,
                                  float** devfreQ, float** devsigP, int cSearch)
{
    (void)cSearch;
    THX_DEV_SET(gpuIdx);
    float** all[5] = {devdatP, devctfP, devdefO, devfreQ, devsigP};
    for (float** p : all)
        if (p && *p) {
            THX_HIP(hipFree(*p));
            *p = nullptr;
        }
    return THX_OK;
}

extern "C" int thx_ExpectLocalHostA(int gpuIdx, float** wC, float** wR, float** wT, float** wD,
                                    double** oldR, double** oldT, double** oldD, double** trans,
                                    double** rot, double** dpara, int mR, int mT, int mD,
                                    int cSearch)
{
    THX_CHECK_ARG(wC && wR && wT && wD && oldR && oldT && oldD && trans && rot && dpara &&
                      mR > 0 && mT > 0,
                  "thx_ExpectLocalHostA: bad arguments");
    THX_DEV_SET(gpuIdx);
    const int nD = cSearch && mD > 0 ? mD : 1;
    THX_HIP(hipHostMalloc(reinterpret_cast<void**>(wC), sizeof(float)));
    THX_HIP(hipHostMalloc(reinterpret_cast<void**>(wR), sizeof(float) * mR));
    THX_HIP(hipHostMalloc(reinterpret_cast<void**>(wT), sizeof(float) * mT));
    THX_HIP(hipHostMalloc(reinterpret_cast<void**>(wD), sizeof(float) * nD));
    THX_HIP(hipHostMalloc(reinterpret_cast<void**>(oldR), sizeof(double) * mR));
    THX_HIP(hipHostMalloc(reinterpret_cast<void**>(oldT), sizeof(double) * mT));
    THX_HIP(hipHostMalloc(reinterpret_cast<void**>(oldD), sizeof(double) * nD));
    THX_HIP(hipHostMalloc(reinterpret_cast<void**>(trans), sizeof(double) * 2 * mT));
    THX_HIP(hipHostMalloc(reinterpret_cast<void**>(rot), sizeof(double) * 4 * mR));
    THX_HIP(hipHostMalloc(reinterpret_cast<void**>(dpara), sizeof(double) * nD));
    return THX_OK;
}

extern "C" int thx_ExpectLocalHostF(int gpuIdx, float** wC, float** wR, float** wT, float** wD,
                                    double** oldR, double** oldT, double** oldD, double** trans,
                                    double** rot, double** dpara, int cSearch)
{
    (void)cSearch;
    THX_DEV_SET(gpuIdx);
    void** all[10] = {(void**)wC, (void**)wR, (void**)wT, (void**)wD, (void**)oldR,
                      (void**)oldT, (void**)oldD, (void**)trans, (void**)rot, (void**)dpara};
    for (void** p : all)
        if (p && *p) {
            THX_HIP(hipHostFree(*p));
            *p = nullptr;
        }
    return THX_OK;
}

// ManagedArrayTexture::Init + ExpectLocalV3D
extern "C" int thx_tex_create(int mode, int vdim, int gpuIdx, void** mgr)
{
    THX_CHECK_ARG(mgr && vdim > 0 && vdim % 2 == 0, "thx_tex_create: bad arguments");
    THX_CHECK_ARG(mode == 0 || mode == 1, "thx_tex_create: mode must be MODE_2D (0) or MODE_3D (1)");
    THX_DEV_SET(gpuIdx);
    Tex* t = new Tex;
    t->vdim = vdim;
    t->gpu = gpuIdx;
    t->mode = mode;
    const size_t dimSize = (size_t)(vdim / 2 + 1) * vdim * (mode == 1 ? vdim : 1);
    if (hipMalloc(&t->vol, sizeof(float) * 2 * dimSize) != hipSuccess) {
        delete t;
        thx::set_error("thx_tex_create: device allocation failed");
        return THX_ERR_NOMEM;
    }
    *mgr = t;
    return THX_OK;
}

extern "C" int thx_tex_destroy(void* mgr)
{
    Tex* t = static_cast<Tex*>(mgr);
    if (!t) return THX_OK;
    THX_DEV_SET(t->gpu);
    if (t->vol) THX_HIP(hipFree(t->vol));
    delete t;
    return THX_OK;
}

extern "C" int thx_ExpectLocalV3D(int gpuIdx, void* mgr, const float* volume, int vdim)
{
    Tex* t = static_cast<Tex*>(mgr);
    THX_CHECK_ARG(t && volume && vdim == t->vdim && gpuIdx == t->gpu && t->mode == 1,
                  "thx_ExpectLocalV3D: volume handle / size / device / mode mismatch");
    THX_DEV_SET(gpuIdx);
    const size_t dimSize = (size_t)(vdim / 2 + 1) * vdim * vdim;
    THX_HIP(hipMemcpy(t->vol, volume, sizeof(float) * 2 * dimSize, hipMemcpyHostToDevice));
    return THX_OK;
}

// ExpectLocalV2D (Interface.h:40-43): one class image, dimSize = (vdim/2+1) vdim
extern "C" int thx_ExpectLocalV2D(int gpuIdx, void* mgr, const float* volume, int dimSize)
{
    Tex* t = static_cast<Tex*>(mgr);
    THX_CHECK_ARG(t && volume && t->mode == 0 && gpuIdx == t->gpu &&
                      (long)dimSize == (long)(t->vdim / 2 + 1) * t->vdim,
                  "thx_ExpectLocalV2D: image handle / size / device / mode mismatch");
    THX_DEV_SET(gpuIdx);
    THX_HIP(hipMemcpy(t->vol, volume, sizeof(float) * 2 * (size_t)dimSize, hipMemcpyHostToDevice));
    return THX_OK;
}

// ManagedCalPoint::Init (mode, searchType, gpu, mLR, mLT, mLD, nPxl)
extern "C" int thx_calpoint_create(int mode, int searchType, int gpuIdx, int mR, int mT, int mD,
                                   int npxl, void** mcp)
{
    THX_CHECK_ARG(mcp && mR > 0 && mT > 0 && npxl > 0, "thx_calpoint_create: bad arguments");
    THX_CHECK_ARG(mode == 0 || mode == 1, "thx_calpoint_create: mode must be 0 (2D) or 1 (3D)");
    THX_CHECK_ARG(searchType != 2 || (mD >= 1 && (long)mT * mD <= 1024),
                  "thx_calpoint_create: CTF search needs 1 <= mD, mT * mD <= 1024");
    THX_DEV_SET(gpuIdx);
    CalPoint* c = new CalPoint;
    c->gpu = gpuIdx;
    c->mR = mR;
    c->mT = mT;
    c->npxl = npxl;
    c->cs = searchType == 2;
    c->mD = c->cs ? mD : 1;
    c->mode = mode;
    int st = THX_OK;
    auto chk = [&](hipError_t e) {
        if (e != hipSuccess && st == THX_OK) {
            thx::set_error("thx_calpoint_create: %s", hipGetErrorString(e));
            st = THX_ERR_NOMEM;
        }
    };
    chk(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    chk(hipMalloc(&c->quat, sizeof(double) * 4 * mR));
    chk(hipMalloc(&c->trans, sizeof(double) * 2 * mT));
    chk(hipMalloc(&c->pR, sizeof(double) * mR));
    chk(hipMalloc(&c->pT, sizeof(double) * mT));
    chk(hipMalloc(&c->pC, sizeof(double)));
    chk(hipMalloc(&c->wC, sizeof(float)));
    chk(hipMalloc(&c->wR, sizeof(float) * mR));
    chk(hipMalloc(&c->wT, sizeof(float) * mT));
    chk(hipMalloc(&c->base, sizeof(float)));
    // the tile order of a pixel set has at most ~1.25 npxl + 16 entries
    const int ordCap = (npxl * 2 + 31) / 16 * 16;
    chk(hipMalloc(&c->order, sizeof(int) * ordCap));
    c->wsBytes = mode == 1 ? thx_local_phase_workspace(1, mR, mT * c->mD, ordCap > npxl ? ordCap : npxl)
                           : thx_local_phase2d_d_workspace(1, mR, mT, c->mD);
    chk(hipMalloc(&c->ws, c->wsBytes));
    if (mode == 0) chk(hipMalloc(&c->rot2, sizeof(double) * 2 * mR));
    if (c->cs) {
        chk(hipMalloc(&c->dP, sizeof(double) * c->mD));
        chk(hipMalloc(&c->pD, sizeof(double) * c->mD));
        chk(hipMalloc(&c->ctfD, sizeof(float) * c->mD * npxl));
        chk(hipMalloc(&c->wD, sizeof(float) * c->mD));
    }
    *mcp = c;
    return st;
}

extern "C" int thx_calpoint_destroy(void* mcp)
{
    CalPoint* c = static_cast<CalPoint*>(mcp);
    if (!c) return THX_OK;
    THX_DEV_SET(c->gpu);
    void* all[] = {c->quat, c->trans, c->pR, c->pT, c->pC, c->wC, c->wR, c->wT, c->base, c->order,
                   c->ws, c->dP, c->pD, c->ctfD, c->wD, c->rot2};
    for (void* p : all)
        if (p) (void)hipFree(p);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return THX_OK;
}

extern "C" int thx_ExpectLocalRTD(int gpuIdx, void* mcp, const double* oldR, const double* oldT,
                                  const double* oldD, const double* trans, const double* rot,
                                  const double* dpara)
{
    CalPoint* c = static_cast<CalPoint*>(mcp);
    THX_CHECK_ARG(c && oldR && oldT && trans && rot && gpuIdx == c->gpu &&
                      (!c->cs || (oldD && dpara)),
                  "thx_ExpectLocalRTD: bad arguments");
    if (c->cs) {
        THX_DEV_SET(gpuIdx);
        THX_HIP(hipMemcpyAsync(c->dP, dpara, sizeof(double) * c->mD, hipMemcpyHostToDevice, c->stream));
        THX_HIP(hipMemcpyAsync(c->pD, oldD, sizeof(double) * c->mD, hipMemcpyHostToDevice, c->stream));
    }
    THX_DEV_SET(gpuIdx);
    THX_HIP(hipMemcpyAsync(c->pR, oldR, sizeof(double) * c->mR, hipMemcpyHostToDevice, c->stream));
    THX_HIP(hipMemcpyAsync(c->pT, oldT, sizeof(double) * c->mT, hipMemcpyHostToDevice, c->stream));
    THX_HIP(hipMemcpyAsync(c->trans, trans, sizeof(double) * 2 * c->mT, hipMemcpyHostToDevice, c->stream));
    THX_HIP(hipMemcpyAsync(c->quat, rot, sizeof(double) * 4 * c->mR, hipMemcpyHostToDevice, c->stream));
    if (c->mode == 0) {
        // 2D: rotation k is (r(k, 0), r(k, 1)) = (cos, sin) of the particle's
        // quaternion row (Particle::rot(dmat22&), src/Particle.cpp:850-854), as
        // Optimiser packs it (4 doubles per rotation, src/Optimiser.cpp:
        // 2468-2476); cuthunder's 2D RTD copies 2 nR doubles and reads them with
        // stride 2 (gpu/src/cuthunder.cu:2700-2717, Kernel.cu:762) -- quirk q9,
        // not replicated
        hipLaunchKernelGGL(k_rot2_from_quat, dim3(thx::cdiv(c->mR, 256)), dim3(256), 0, c->stream,
                           c->quat, c->mR, c->rot2);
        THX_LAUNCH_CHECK();
    }
    return THX_OK;
}

extern "C" int thx_ExpectLocalPreI3D(int gpuIdx, int datShift, void* mgr, void* mcp,
                                     const float* devdefO, const float* devfreQ,
                                     const int* deviCol, const int* deviRow, float phaseShift,
                                     float conT, float k1, float k2, int pf, int idim, int vdim,
                                     int npxl, int interp)
{
    CalPoint* c = static_cast<CalPoint*>(mcp);
    const Tex* t = static_cast<const Tex*>(mgr);
    THX_CHECK_ARG(c && t && deviCol && deviRow && gpuIdx == c->gpu && npxl == c->npxl &&
                      c->mode == 1 && t->mode == 1 && vdim == t->vdim && vdim == pf * idim,
                  "thx_ExpectLocalPreI3D: bad arguments");
    THX_CHECK_ARG(interp == 1, "thx_ExpectLocalPreI3D: only LINEAR_INTERP (1) is supported");
    THX_CHECK_ARG(!c->cs || (devdefO && devfreQ && datShift >= 0),
                  "thx_ExpectLocalPreI3D: a CTF search needs devdefO and devfreQ");
    THX_DEV_SET(gpuIdx);
    if (c->cs) {
        hipLaunchKernelGGL(k_calpoint_ctf, dim3(thx::cdiv(npxl, 256) > 16 ? 16 : thx::cdiv(npxl, 256),
                                                c->mD),
                           dim3(256), 0, c->stream, devdefO + (size_t)datShift * npxl, devfreQ,
                           c->dP, phaseShift, conT, k1, k2, npxl, c->ctfD);
        THX_LAUNCH_CHECK();
    }
    if (c->boundCol != deviCol) {
        // the pixel set's local-phase visiting order, once per calpoint and set
        std::vector<int> hc(npxl), hr(npxl);
        THX_HIP(hipMemcpy(hc.data(), deviCol, sizeof(int) * npxl, hipMemcpyDeviceToHost));
        THX_HIP(hipMemcpy(hr.data(), deviRow, sizeof(int) * npxl, hipMemcpyDeviceToHost));
        int nOrd = 0;
        THX_RET(thx_pixel_tile_order(hc.data(), hr.data(), npxl, 0, nullptr, &nOrd));
        const int ordCap = (npxl * 2 + 31) / 16 * 16;
        THX_CHECK_ARG(nOrd <= ordCap, "thx_ExpectLocalPreI3D: tile order too long");
        std::vector<int> ord(nOrd);
        THX_RET(thx_pixel_tile_order(hc.data(), hr.data(), npxl, nOrd, ord.data(), &nOrd));
        THX_HIP(hipMemcpy(c->order, ord.data(), sizeof(int) * nOrd, hipMemcpyHostToDevice));
        c->nOrd = nOrd;
        c->boundCol = deviCol;
    }
    c->tex = t;
    c->iCol = deviCol;
    c->iRow = deviRow;
    c->pf = pf;
    c->idim = idim;
    c->vdim = vdim;
    return THX_OK;
}

// ExpectLocalPreI2D (Interface.h:89-105; cuthunder.cu:2762-2825): binds the
// class image, pixel set and geometry (the 2D phase projects on the fly from
// the image in LDS); with CTF search the calpoint's CTF per defocus sample
// (kernel_CalCTFL from devdefO / devfreQ, as ExpectLocalPreI3D).
extern "C" int thx_ExpectLocalPreI2D(int gpuIdx, int datShift, void* mgr, void* mcp,
                                     const float* devdefO, const float* devfreQ,
                                     const int* deviCol, const int* deviRow, float phaseShift,
                                     float conT, float k1, float k2, int pf, int idim, int vdim,
                                     int npxl, int interp)
{
    CalPoint* c = static_cast<CalPoint*>(mcp);
    const Tex* t = static_cast<const Tex*>(mgr);
    THX_CHECK_ARG(c && t && deviCol && deviRow && gpuIdx == c->gpu && npxl == c->npxl &&
                      c->mode == 0 && t->mode == 0 && vdim == t->vdim && vdim == pf * idim,
                  "thx_ExpectLocalPreI2D: bad arguments");
    THX_CHECK_ARG(interp == 1, "thx_ExpectLocalPreI2D: only LINEAR_INTERP (1) is supported");
    THX_CHECK_ARG(!c->cs || (devdefO && devfreQ && datShift >= 0),
                  "thx_ExpectLocalPreI2D: a CTF search needs devdefO and devfreQ");
    THX_DEV_SET(gpuIdx);
    if (c->cs) {
        hipLaunchKernelGGL(k_calpoint_ctf, dim3(thx::cdiv(npxl, 256) > 16 ? 16 : thx::cdiv(npxl, 256),
                                                c->mD),
                           dim3(256), 0, c->stream, devdefO + (size_t)datShift * npxl, devfreQ,
                           c->dP, phaseShift, conT, k1, k2, npxl, c->ctfD);
        THX_LAUNCH_CHECK();
    }
    c->tex = t;
    c->iCol = deviCol;
    c->iRow = deviRow;
    c->pf = pf;
    c->idim = idim;
    c->vdim = vdim;
    return THX_OK;
}

extern "C" int thx_ExpectLocalM(int gpuIdx, int datShift, void* mcp, const float* devdatP,
                                const float* devctfP, const float* devsigP, float* wC, float* wR,
                                float* wT, float* wD, double oldC, int npxl)
{
    CalPoint* c = static_cast<CalPoint*>(mcp);
    THX_CHECK_ARG(c && c->tex && devdatP && devctfP && devsigP && wC && wR && wT &&
                      gpuIdx == c->gpu && npxl == c->npxl && datShift >= 0 && (!c->cs || wD),
                  "thx_ExpectLocalM: bad arguments (ExpectLocalPreI3D must come first)");
    THX_DEV_SET(gpuIdx);
    const size_t off = (size_t)datShift * npxl;
    THX_HIP(hipMemcpyAsync(c->pC, &oldC, sizeof(double), hipMemcpyHostToDevice, c->stream));
    if (c->mode == 0 && c->cs) {
        // the 2D (r, t, d) phase (kernel_logDataVSLC + kernel_UpdateWLC on the
        // 2D projections)
        THX_RET(thx_local_phase2d_d(c->tex->vol, c->vdim, c->pf, nullptr, c->rot2, c->mR,
                                    c->trans, c->mT, c->mD, c->pC, c->pR, c->pT, c->pD,
                                    devdatP + 2 * off, c->ctfD, devsigP + off, c->iCol, c->iRow,
                                    npxl, c->idim, 1, c->wC, c->wR, c->wT, c->wD, c->base, nullptr,
                                    c->ws, c->wsBytes, c->stream));
        THX_HIP(hipMemcpyAsync(wC, c->wC, sizeof(float), hipMemcpyDeviceToHost, c->stream));
        THX_HIP(hipMemcpyAsync(wR, c->wR, sizeof(float) * c->mR, hipMemcpyDeviceToHost, c->stream));
        THX_HIP(hipMemcpyAsync(wT, c->wT, sizeof(float) * c->mT, hipMemcpyDeviceToHost, c->stream));
        THX_HIP(hipMemcpyAsync(wD, c->wD, sizeof(float) * c->mD, hipMemcpyDeviceToHost, c->stream));
        THX_HIP(hipStreamSynchronize(c->stream));
        return THX_OK;
    }
    if (c->mode == 0) {
        // the 2D phase (kernel_logDataVSL + kernel_UpdateWL on the 2D
        // projections, cuthunder.cu:2915-3140)
        THX_RET(thx_local_phase2d(c->tex->vol, c->vdim, c->pf, nullptr, c->rot2, c->mR, c->trans,
                                  c->mT, c->pC, c->pR, c->pT, devdatP + 2 * off, devctfP + off,
                                  devsigP + off, c->iCol, c->iRow, npxl, c->idim, 1, c->wC, c->wR,
                                  c->wT, c->base, nullptr, c->ws, c->wsBytes, c->stream));
        THX_HIP(hipMemcpyAsync(wC, c->wC, sizeof(float), hipMemcpyDeviceToHost, c->stream));
        THX_HIP(hipMemcpyAsync(wR, c->wR, sizeof(float) * c->mR, hipMemcpyDeviceToHost, c->stream));
        THX_HIP(hipMemcpyAsync(wT, c->wT, sizeof(float) * c->mT, hipMemcpyDeviceToHost, c->stream));
        THX_HIP(hipStreamSynchronize(c->stream));
        if (wD) wD[0] = (float)(oldC * (double)wC[0]);
        return THX_OK;
    }
    if (c->cs) {
        // kernel_logDataVSLC + kernel_UpdateWLC (cuthunder.cu:2915-3140)
        THX_RET(thx_local_phase_d(nullptr, c->tex->vol, 0, c->vdim, c->pf, c->quat, c->mR,
                                  c->trans, c->mT, c->mD, c->pC, c->pR, c->pT, c->pD,
                                  devdatP + 2 * off, c->ctfD, devsigP + off, c->iCol, c->iRow,
                                  c->order, c->nOrd, npxl, c->idim, 1, c->wC, c->wR, c->wT, c->wD,
                                  c->base, nullptr, c->ws, c->wsBytes, c->stream));
        THX_HIP(hipMemcpyAsync(wC, c->wC, sizeof(float), hipMemcpyDeviceToHost, c->stream));
        THX_HIP(hipMemcpyAsync(wR, c->wR, sizeof(float) * c->mR, hipMemcpyDeviceToHost, c->stream));
        THX_HIP(hipMemcpyAsync(wT, c->wT, sizeof(float) * c->mT, hipMemcpyDeviceToHost, c->stream));
        THX_HIP(hipMemcpyAsync(wD, c->wD, sizeof(float) * c->mD, hipMemcpyDeviceToHost, c->stream));
        THX_HIP(hipStreamSynchronize(c->stream));
        return THX_OK;
    }
    THX_RET(thx_local_phase(c->tex->vol, 0, c->vdim, c->pf, c->quat, c->mR, c->trans, c->mT, c->pC,
                            c->pR, c->pT, devdatP + 2 * off, devctfP + off, devsigP + off, c->iCol,
                            c->iRow, c->order, c->nOrd, npxl, c->idim, 1, c->wC, c->wR, c->wT,
                            c->base, nullptr, c->ws, c->wsBytes, c->stream));
    THX_HIP(hipMemcpyAsync(wC, c->wC, sizeof(float), hipMemcpyDeviceToHost, c->stream));
    THX_HIP(hipMemcpyAsync(wR, c->wR, sizeof(float) * c->mR, hipMemcpyDeviceToHost, c->stream));
    THX_HIP(hipMemcpyAsync(wT, c->wT, sizeof(float) * c->mT, hipMemcpyDeviceToHost, c->stream));
    THX_HIP(hipStreamSynchronize(c->stream));   // the reference's sync (cuthunder.cu:3140)
    // nD = 1 (wD prior 1): wD(0) = sum s wC(0) wR(r) wT(t) = oldC * wC
    // (src/Optimiser.cpp:1399-1402)
    if (wD) wD[0] = (float)(oldC * (double)wC[0]);
    return THX_OK;
}
