// interface_restated.h -- TEST-ONLY restatement of the hot-path prototypes of
// THUNDER's GPU plugin boundary, gpu/interface/Interface.h (line numbers
// below), over the restated types of thunder_restated.h.  The INTEGRATION.md
// forwards are compiled with -Werror=missing-declarations after this header:
// a forward whose signature drifts from the reference's declaration is a new
// overload without a previous declaration and fails the build
// (tests/test_integration.py).  Out-of-scope Interface.h entries
// (PrepareTF, Expose*, TranslateI*, ReMask, GCTFinit, ExpectPrecal) are not
// restated: the drop-in keeps the reference's own bodies for them.
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
