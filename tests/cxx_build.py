"""Builds tests/cxx/adapter_test (the ORB_SLAM2:: drop-in exercised through its
reference-shaped signatures) against liborbx.so and the test-only cv mock."""
import subprocess
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def build_adapter_test() -> Path:
    out = Path(tempfile.mkdtemp(prefix="orbx_cxx_")) / "adapter_test"
    lib_dir = ROOT / "orb_slam_2_ros_amd"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", f"-I{ROOT / 'include'}",
                    f"-I{ROOT / 'tests' / 'cxx' / 'cv_mock'}", str(ROOT / "tests" / "cxx" / "adapter_test.cpp"),
                    f"-L{lib_dir}", "-lorbx", f"-Wl,-rpath,{lib_dir}", "-o", str(out)], check=True)
    return out
