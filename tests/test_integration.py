"""The INTEGRATION.md forwards (gpu/interface/Interface.cpp bodies and the
handle classes) compile against a restatement of the THUNDER types they touch
(tests/integration/thunder_restated.h) and MPICH's mpi.h, and link against
libthunder_amd.so with every symbol resolved: the drop-in boundary cannot
drift from include/thunder_amd.h.  CPU only (nothing is called on a GPU)."""
import os
import re
import shutil
import subprocess

import pytest

from thunder_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPI_INC = "/opt/conda/include"
MPI_LIB = "/opt/conda/lib"


# The Interface.h functions (gpu/interface/Interface.h:16-528) that THUNDER's
# src/ calls, with their overload counts; ExpectPrecal (:166) is the one
# declaration nothing in src/ calls.
SRC_CALLED = {
    "getAviDevice": 1, "ExpectPreidx": 1, "ExpectPrefre": 1, "ExpectLocalIn": 1,
    "ExpectLocalV2D": 1, "ExpectLocalV3D": 1, "ExpectLocalP": 1, "ExpectLocalHostA": 1,
    "ExpectLocalRTD": 1, "ExpectLocalPreI2D": 1, "ExpectLocalPreI3D": 1, "ExpectLocalM": 1,
    "ExpectLocalHostF": 1, "ExpectLocalFin": 1, "ExpectFreeIdx": 1, "ExpectGlobal2D": 1,
    "ExpectRotran": 1, "ExpectProject": 1, "ExpectGlobal3D": 1, "InsertI2D": 1, "InsertFT": 2,
    "PrepareTF": 1, "ExposePT2D": 1, "ExposePT": 1, "ExposeWT2D": 2, "AllocDevicePoint": 1,
    "HostDeviceInit": 1, "ExposeC": 1, "ExposeForConvC": 1, "ExposeWC": 1,
    "FreeDevHostPoint": 1, "ExposeWT": 2, "ExposePF2D": 1, "ExposePFW": 1, "ExposePF": 1,
    "ExposeCorrF2D": 1, "ExposeCorrF": 2, "TranslateI2D": 1, "TranslateI": 1, "ReMask": 1,
    "GCTFinit": 1,
}


def blocks():
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    out = []
    for name in ("Interface.cpp", "handles"):
        m = re.search(rf"// BEGIN {re.escape(name)}\n(.*?)// END {re.escape(name)}", txt, re.S)
        assert m, f"INTEGRATION.md has no '{name}' block"
        out.append(m.group(1))
    return out


def test_integration_blocks_present():
    iface, handles = blocks()
    # every Interface.h entry point src/ calls is forwarded, overloads included
    for fn, n in SRC_CALLED.items():
        assert len(re.findall(rf"^void {fn}\(", iface, re.M)) == n, fn
    assert "thx_tex_create" in handles and "thx_calpoint_create" in handles


@pytest.mark.skipif(not (os.path.exists(os.path.join(MPI_INC, "mpi.h")) and shutil.which("g++")),
                    reason="needs g++ and MPICH's mpi.h")
def test_forwards_compile_and_link(tmp_path):
    lib = build.build()
    iface, handles = blocks()
    src = tmp_path / "Interface_thx.cpp"
    # the reference's prototypes first: -Werror=missing-declarations turns any
    # forward whose signature differs from Interface.h's into a build error
    src.write_text('#include "interface_restated.h"\n' + iface + "\n" + handles)
    out = tmp_path / "libinterface_thx.so"
    cmd = ["g++", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Werror", "-Wno-unused-parameter",
           "-Werror=missing-declarations",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "tests", "integration"),
           "-I", MPI_INC, str(src), "-o", str(out), "-Wl,--no-undefined",
           "-L", os.path.dirname(lib), "-lthunder_amd", os.path.join(MPI_LIB, "libmpi.so"),
           f"-Wl,-rpath,{os.path.dirname(lib)}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    nm = subprocess.run(["nm", "-D", "--defined-only", "-C", str(out)], capture_output=True,
                        text=True).stdout
    for sig in ("ExpectLocalM(int, int, ManagedCalPoint*", "InsertFT(Volume&, Volume&, double*, int*",
                "ManagedCalPoint::Init(int, int, int, int, int, int, int)", "getAviDevice(",
                "InsertI2D(Complex*, float*, double*, int*, ompi_communicator_t*&",
                "ExpectGlobal2D(Complex*, Complex*, float*",
                "ExposeWC(int, Volume&, Complex*, float*, float*, float*, float*, float*, int*, int*, "
                "void**, float&", "ExposeCorrF(int, Volume&, Volume&, float*, float)",
                "ReMask(std::vector<Image, std::allocator<Image> >&", "PrepareTF(int, Volume&, Volume&"):
        assert sig.split("ompi")[0] in nm, sig
    # every forward is a defined, exported symbol of the drop-in library
    defined = re.findall(r"^[0-9a-f]+ T (\w+)\(", nm, re.M)
    for fn, n in SRC_CALLED.items():
        assert defined.count(fn) == n, (fn, defined.count(fn))


def test_drifted_forward_fails_to_compile(tmp_path):
    """The guard itself: a forward with one argument type changed from
    Interface.h's declaration does not compile."""
    if not (os.path.exists(os.path.join(MPI_INC, "mpi.h")) and shutil.which("g++")):
        pytest.skip("needs g++ and MPICH's mpi.h")
    src = tmp_path / "drift.cpp"
    src.write_text('#include "interface_restated.h"\n'
                   "void ExpectFreeIdx(int gpuIdx, int** deviCol, long** deviRow) {}\n")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Werror=missing-declarations",
                        "-I", os.path.join(ROOT, "tests", "integration"), "-I", MPI_INC, str(src)],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "missing-declarations" in r.stderr
