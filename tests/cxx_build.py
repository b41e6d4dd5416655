"""Builds tests/cxx/adapter_test (the ORB_SLAM2:: drop-in exercised through its
reference-shaped signatures) against liborbx.so and the test-only cv mock."""
import subprocess
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def build_adapter_test(out: Path = None) -> Path:
    out = Path(out) if out is not None else Path(tempfile.mkdtemp(prefix="orbx_cxx_")) / "adapter_test"
    out.parent.mkdir(parents=True, exist_ok=True)
    lib_dir = ROOT / "orb_slam_2_ros_amd"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", f"-I{ROOT / 'include'}",
                    f"-I{ROOT / 'tests' / 'cxx' / 'cv_mock'}", str(ROOT / "tests" / "cxx" / "adapter_test.cpp"),
                    f"-L{lib_dir}", "-lorbx", f"-Wl,-rpath,{lib_dir}", "-o", str(out)], check=True)
    return out


FORWARDERS = ["integration/ORBmatcher_orbx.cc", "integration/Optimizer_orbx.cc",
              "integration/KeyFrameDatabase_orbx.cc", "integration/Frame_orbx.cc", "integration/LocalMapping_orbx.cc",
              "tests/cxx/orbslam_mock/mock_impl.cpp", "tests/cxx/forwarders_test.cpp"]


def build_forwarders_test(backend: str) -> Path:
    """tests/cxx/forwarders_test: the reference-side forwarders of integration/
    compiled against the test stand-ins of the reference headers.  backend
    "liborbx" links the product library (the GPU run); "oracle" answers the
    orbx_* calls with the CPU oracle (tests/cxx/orbx_oracle_shim.cpp), so the
    forwarders' own logic is checked without a GPU."""
    out = Path(tempfile.mkdtemp(prefix="orbx_fwd_")) / f"forwarders_test_{backend}"
    lib_dir, oracle_dir = ROOT / "orb_slam_2_ros_amd", ROOT / "oracle"
    srcs = [str(ROOT / s) for s in FORWARDERS]
    if backend == "oracle":
        srcs.append(str(ROOT / "tests" / "cxx" / "orbx_oracle_shim.cpp"))
        libs = []
    elif backend == "liborbx":
        libs = [f"-L{lib_dir}", "-lorbx", f"-Wl,-rpath,{lib_dir}"]
    else:
        raise ValueError(backend)
    inc = [ROOT / "integration", ROOT / "tests" / "cxx" / "orbslam_mock", ROOT / "tests" / "cxx" / "cv_mock",
           ROOT / "include", oracle_dir]
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", *[f"-I{i}" for i in inc], *srcs,
                    *libs, f"-L{oracle_dir}", "-lorbx_oracle", f"-Wl,-rpath,{oracle_dir}", "-o", str(out)],
                   check=True)
    return out
