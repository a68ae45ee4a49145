// thunder_restated.h -- TEST-ONLY restatement of the THUNDER declarations the
// INTEGRATION.md forwards touch, so tests/test_integration.py can compile and
// link them against libthunder_amd.so without the reference tree (whose
// headers need Boost, absent here).  Layouts follow the reference's
// single-precision build: RFLOAT = float, Complex = {float dat[2]}
// (include/Precision.h:64-106, include/Complex.h), CTFAttr
// (include/Database.h:302), Volume's / Image's FT and RL storage and size
// accessors (include/Image/Volume.h, Image.h), TabFunction's table accessors,
// Eigen's vec as far as data() / size(), and the public Init signatures of
// ManagedArrayTexture / ManagedCalPoint (gpu/include/ManagedArrayTexture.h:17,
// gpu/include/ManagedCalPoint.h:16-22) plus the one member / accessor the
// integration adds to each.
#pragma once
#include <mpi.h>

#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float RFLOAT;
struct Complex {
    RFLOAT dat[2];
};
#define REAL(x) ((x).dat[0])
inline Complex COMPLEX(RFLOAT re, RFLOAT im)
{
    Complex c;
    c.dat[0] = re;
    c.dat[1] = im;
    return c;
}
#define REPORT_ERROR(msg) std::fprintf(stderr, "ERROR: %s\n", (msg))

struct CTFAttr {
    RFLOAT voltage, defocusU, defocusV, defocusTheta, Cs, amplitudeContrast, phaseShift;
};

// Volume / Image: the half-complex FT array (operator[]) and the real-space
// array (operator()) are separate buffers, as ImageBase keeps _dataFT and
// _dataRL (src/Image/Volume.cpp:89-119, src/Image/Image.cpp:81-99)
class Volume {
public:
    Volume(int n) : _n(n), _d((size_t)(n / 2 + 1) * n * n), _r((size_t)n * n * n) {}
    Complex& operator[](size_t i) { return _d[i]; }
    RFLOAT& operator()(size_t i) { return _r[i]; }
    long nSlcFT() const { return _n; }
    long nSlcRL() const { return _n; }
    size_t sizeFT() const { return _d.size(); }

private:
    int _n;
    std::vector<Complex> _d;
    std::vector<RFLOAT> _r;
};

class Image {
public:
    Image(int n) : _n(n), _d((size_t)(n / 2 + 1) * n), _r((size_t)n * n) {}
    Complex& operator[](size_t i) { return _d[i]; }
    RFLOAT& operator()(size_t i) { return _r[i]; }
    long nRowFT() const { return _n; }
    long nRowRL() const { return _n; }

private:
    int _n;
    std::vector<Complex> _d;
    std::vector<RFLOAT> _r;
};

// TabFunction's table accessors (include/TabFunction.h:61-63)
class TabFunction {
public:
    RFLOAT* getData() const { return _tab; }
    RFLOAT getStep() const { return _s; }

private:
    RFLOAT* _tab = nullptr;
    RFLOAT _s = 1e-5f;
};

// vec = Eigen::Matrix<RFLOAT, Dynamic, 1> (include/Typedef.h:54): the two
// members the forwards use
class vec {
public:
    const RFLOAT* data() const { return _v.data(); }
    long size() const { return (long)_v.size(); }

private:
    std::vector<RFLOAT> _v;
};

class ManagedArrayTexture {
public:
    ~ManagedArrayTexture();
    void Init(int mode, int vdim, int gpuIdx);
    void* thx() const { return _thx; }

private:
    void* _thx = nullptr;
};

class ManagedCalPoint {
public:
    ~ManagedCalPoint();
    void Init(int mode, int cSearch, int gpuIdx, int nR, int nT, int mD, int npxl);
    void* thx() const { return _thx; }

private:
    void* _thx = nullptr;
};
