// interface_restated.h -- TEST-ONLY restatement of the prototypes of
// THUNDER's GPU plugin boundary, gpu/interface/Interface.h (line numbers
// below), over the restated types of thunder_restated.h.  The INTEGRATION.md
// forwards are compiled with -Werror=missing-declarations after this header:
// a forward whose signature drifts from the reference's declaration is a new
// overload without a previous declaration and fails the build
// (tests/test_integration.py).  Every Interface.h function src/ calls is
// restated; ExpectPrecal (:166), which nothing in src/ calls, is not.
#pragma once
#include "thunder_restated.h"

void getAviDevice(std::vector<int>& gpus);                                       // :16
void ExpectPreidx(int gpuIdx, int** deviCol, int** deviRow, int* iCol, int* iRow,
                  int npxl);                                                     // :18-23
void ExpectPrefre(int gpuIdx, RFLOAT** devfreQ, RFLOAT* freQ, int npxl);         // :26-29
void ExpectLocalIn(int gpuIdx, Complex** devdatP, RFLOAT** devctfP, RFLOAT** devdefO,
                   RFLOAT** devsigP, int nPxl, int cpyNumL, int searchType);     // :31-38
void ExpectLocalV2D(int gpuIdx, ManagedArrayTexture* mgr, Complex* volume,
                    int dimSize);                                                // :40-43
void ExpectLocalV3D(int gpuIdx, ManagedArrayTexture* mgr, Complex* volume,
                    int vdim);                                                   // :45-48
void ExpectLocalP(int gpuIdx, Complex* devdatP, RFLOAT* devctfP, RFLOAT* devdefO,
                  RFLOAT* devsigP, Complex* datP, RFLOAT* ctfP, RFLOAT* defO, RFLOAT* sigP,
                  int threadId, int imgId, int npxl, int cSearch);               // :50-62
void ExpectLocalHostA(int gpuIdx, RFLOAT** wC, RFLOAT** wR, RFLOAT** wT, RFLOAT** wD,
                      double** oldR, double** oldT, double** oldD, double** trans,
                      double** rot, double** dpara, int mR, int mT, int mD,
                      int cSearch);                                              // :64-78
void ExpectLocalRTD(int gpuIdx, ManagedCalPoint* mcp, double* oldR, double* oldT,
                    double* oldD, double* trans, double* rot, double* dpara);    // :80-87
void ExpectLocalPreI2D(int gpuIdx, int datShift, ManagedArrayTexture* mgr,
                       ManagedCalPoint* mcp, RFLOAT* devdefO, RFLOAT* devfreQ, int* deviCol,
                       int* deviRow, RFLOAT phaseShift, RFLOAT conT, RFLOAT k1, RFLOAT k2,
                       int pf, int idim, int vdim, int npxl, int interp);        // :89-105
void ExpectLocalPreI3D(int gpuIdx, int datShift, ManagedArrayTexture* mgr,
                       ManagedCalPoint* mcp, RFLOAT* devdefO, RFLOAT* devfreQ, int* deviCol,
                       int* deviRow, RFLOAT phaseShift, RFLOAT conT, RFLOAT k1, RFLOAT k2,
                       int pf, int idim, int vdim, int npxl, int interp);        // :107-123
void ExpectLocalM(int gpuIdx, int datShift, ManagedCalPoint* mcp, Complex* devdatP,
                  RFLOAT* devctfP, RFLOAT* devsigP, RFLOAT* wC, RFLOAT* wR, RFLOAT* wT,
                  RFLOAT* wD, double oldC, int npxl);                            // :125-139
void ExpectLocalHostF(int gpuIdx, RFLOAT** wC, RFLOAT** wR, RFLOAT** wT, RFLOAT** wD,
                      double** oldR, double** oldT, double** oldD, double** trans,
                      double** rot, double** dpara, int cSearch);                // :141-152
void ExpectLocalFin(int gpuIdx, Complex** devdatP, RFLOAT** devctfP, RFLOAT** devdefO,
                    RFLOAT** devfreQ, RFLOAT** devsigP, int cSearch);            // :154-160
void ExpectFreeIdx(int gpuIdx, int** deviCol, int** deviRow);                   // :162-164
void ExpectGlobal2D(Complex* vol, Complex* datP, RFLOAT* ctfP, RFLOAT* sigRcpP,
                    double* trans, RFLOAT* wC, RFLOAT* wR, RFLOAT* wT, double* pR,
                    double* pT, double* rot, const int* iCol, const int* iRow, int nK,
                    int nR, int nT, int pf, int interp, int idim, int vdim, int npxl,
                    int imgNum);                                                 // :176-197
void ExpectRotran(Complex* traP, double* trans, double* rot, double* rotMat,
                  const int* iCol, const int* iRow, int nR, int nT, int idim,
                  int npxl);                                                     // :199-208
void ExpectProject(Complex* volume, Complex* rotP, double* rotMat, const int* iCol,
                   const int* iRow, int nR, int pf, int interp, int vdim,
                   int npxl);                                                    // :210-219
void ExpectGlobal3D(Complex* rotP, Complex* traP, Complex* datP, RFLOAT* ctfP,
                    RFLOAT* sigRcpP, RFLOAT* wC, RFLOAT* wR, RFLOAT* wT, double* pR,
                    double* pT, RFLOAT* baseL, int kIdx, int nK, int nR, int nT, int npxl,
                    int imgNum);                                                 // :221-237
void InsertI2D(Complex* F2D, RFLOAT* T2D, double* O2D, int* counter, MPI_Comm& hemi,
               MPI_Comm& slav, Complex* datP, RFLOAT* ctfP, RFLOAT* sigRcpP, RFLOAT* w,
               double* offS, int* nC, double* nR, double* nT, double* nD, CTFAttr* ctfaData,
               const int* iCol, const int* iRow, RFLOAT pixelSize, bool cSearch, int nk,
               int opf, int npxl, int mReco, int idim, int vdim, int imgNum);     // :239-265
void InsertFT(Volume& F3D, Volume& T3D, double* O3D, int* counter, MPI_Comm& hemi,
              MPI_Comm& slav, Complex* datP, RFLOAT* ctfP, RFLOAT* sigRcpP, CTFAttr* ctfaData,
              double* offS, RFLOAT* w, double* nR, double* nT, double* nD, int* nC,
              const int* iCol, const int* iRow, RFLOAT pixelSize, bool cSearch, int opf,
              int npxl, int mReco, int idim, int dimSize, int imgNum);           // :267-292
void InsertFT(Volume& F3D, Volume& T3D, double* O3D, int* counter, MPI_Comm& hemi,
              MPI_Comm& slav, Complex* datP, RFLOAT* ctfP, RFLOAT* sigRcpP, CTFAttr* ctfaData,
              double* offS, RFLOAT* w, double* nR, double* nT, double* nD, const int* iCol,
              const int* iRow, RFLOAT pixelSize, bool cSearch, int opf, int npxl, int mReco,
              int idim, int dimSize, int imgNum);                                // :294-318
void PrepareTF(int gpuIdx, Volume& F3D, Volume& T3D, double* symMat, int nSymmetryElement,
               int maxRadius, int pf);                                           // :320-326
void ExposePT2D(int gpuIdx, RFLOAT* T2D, int maxRadius, int pf, int dim, vec FSC, bool joinHalf,
                const int wienerF);                                              // :328-335
void ExposePT(int gpuIdx, RFLOAT* T3D, int maxRadius, int pf, int dim, vec FSC, bool joinHalf,
              const int wienerF);                                                // :337-344
void ExposeWT2D(int gpuIdx, RFLOAT* T2D, RFLOAT* W2D, TabFunction& kernelRL, RFLOAT nf,
                int maxRadius, int pf, int dim, int maxIter, int minIter, int size); // :346-356
void AllocDevicePoint(int gpuIdx, Complex** dev_C, RFLOAT** dev_W, RFLOAT** dev_T,
                      RFLOAT** dev_tab, RFLOAT** devDiff, RFLOAT** devMax, int** devCount,
                      void** stream, int streamNum, int tabSize, int dim);      // :358-369
void HostDeviceInit(int gpuIdx, Volume& C3D, RFLOAT* W3D, RFLOAT* T3D, RFLOAT* tab,
                    RFLOAT* dev_W, RFLOAT* dev_T, RFLOAT* dev_tab, void** stream, int streamNum,
                    int tabSize, int maxRadius, int pf, int dim);                // :371-384
void ExposeC(int gpuIdx, Volume& C3D, Complex* dev_C, RFLOAT* dev_T, RFLOAT* dev_W,
             void** stream, int streamNum, int dim);                             // :386-393
void ExposeForConvC(int gpuIdx, Volume& C3D, Complex* dev_C, RFLOAT* dev_tab, void** stream,
                    TabFunction& kernelRL, RFLOAT nf, int streamNum, int tabSize, int pf,
                    int size);                                                   // :395-405
void ExposeWC(int gpuIdx, Volume& C3D, Complex* dev_C, RFLOAT* diff, RFLOAT* cmax,
              RFLOAT* dev_W, RFLOAT* devDiff, RFLOAT* devMax, int* devCount, int* counter,
              void** stream, RFLOAT& diffC, int streamNum, int maxRadius, int pf); // :407-421
void FreeDevHostPoint(int gpuIdx, Complex** dev_C, RFLOAT** dev_W, RFLOAT** dev_T,
                      RFLOAT** dev_tab, RFLOAT** devDiff, RFLOAT** devMax, int** devCount,
                      void** stream, Volume& C3D, RFLOAT* volumeW, RFLOAT* volumeT,
                      int streamNum, int dim);                                   // :423-436
void ExposeWT(int gpuIdx, RFLOAT* T3D, RFLOAT* W3D, TabFunction& kernelRL, RFLOAT nf,
              int maxRadius, int pf, int dim, int maxIter, int minIter, int size); // :438-448
void ExposeWT2D(int gpuIdx, RFLOAT* T2D, RFLOAT* W2D, int maxRadius, int pf, int dim); // :450-455
void ExposeWT(int gpuIdx, RFLOAT* T3D, RFLOAT* W3D, int maxRadius, int pf, int dim); // :457-462
void ExposePF2D(int gpuIdx, Image& padDst, Image& padDstR, Image& F2D, RFLOAT* W2D,
                int maxRadius, int pf);                                          // :464-470
void ExposePFW(int gpuIdx, Volume& padDst, Volume& F3D, RFLOAT* W3D, int maxRadius,
               int pf);                                                          // :472-477
void ExposePF(int gpuIdx, Volume& padDst, Volume& padDstR, Volume& F3D, RFLOAT* W3D,
              int maxRadius, int pf);                                            // :479-485
void ExposeCorrF2D(int gpuIdx, Image& imgDst, Volume& dst, RFLOAT* mkbRL, RFLOAT nf); // :487-491
void ExposeCorrF(int gpuIdx, Volume& dst, RFLOAT* mkbRL, RFLOAT nf);            // :493-496
void ExposeCorrF(int gpuIdx, Volume& dstN, Volume& dst, RFLOAT* mkbRL, RFLOAT nf); // :498-502
void TranslateI2D(int gpuIdx, Image& img, double ox, double oy, int r);         // :504-508
void TranslateI(int gpuIdx, Volume& ref, double ox, double oy, double oz, int r); // :510-515
void ReMask(std::vector<Image>& img, RFLOAT maskRadius, RFLOAT pixelSize, RFLOAT ew, int idim,
            int imgNum);                                                         // :517-522
void GCTFinit(std::vector<Image>& img, std::vector<CTFAttr>& ctfAttr, RFLOAT pixelSize,
              int idim, int imgNum);                                             // :524-528
