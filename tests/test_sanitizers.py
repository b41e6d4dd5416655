"""ASan + UBSan on the CPU side, no GPU needed:

- the oracle (oracle/orbx_oracle.cpp) and the product's host plan geometry
  (orb_slam_2_ros_amd/csrc/orbx_plan.h) built with -fsanitize=address,undefined
  and driven over every configuration and edge case the tests use
  (tests/cxx/san_oracle_test.cpp);
- the host side of liborbx's C ABI (every .hip compiled with -Xarch_host
  -fsanitize=..., device code unchanged): argument validation, the error
  strings, DescriptorDistance and both DBoW2 vocabulary loaders on valid and
  malformed files (tests/cxx/san_host_test.cpp).

A sanitizer report makes the driver exit non-zero."""
import os
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
HIPCC = "/opt/rocm/bin/hipcc"
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def test_oracle_and_plan_under_asan_ubsan(tmp_path):
    exe = tmp_path / "san_oracle_test"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-ffp-contract=off", "-fno-omit-frame-pointer",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                    str(ROOT / "tests" / "cxx" / "san_oracle_test.cpp"), str(ROOT / "oracle" / "orbx_oracle.cpp"),
                    "-o", str(exe)], check=True, timeout=600)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=ENV)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "sanitize ok" in r.stdout and "runtime error" not in r.stderr


def test_c_abi_host_side_under_asan_ubsan(tmp_path):
    csrc = ROOT / "orb_slam_2_ros_amd" / "csrc"
    jobs = str(min(8, os.cpu_count() or 2))
    subprocess.run(["make", "-s", "-j", jobs, "-C", str(csrc), "sanitize"], check=True, timeout=900)
    objs = sorted(str(p) for p in (csrc / "_san").glob("*.o"))
    assert len(objs) >= 11
    exe = tmp_path / "san_host_test"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-x", "c++", f"-I{ROOT / 'include'}",
                    "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                    str(ROOT / "tests" / "cxx" / "san_host_test.cpp"), "-x", "none", *objs, "-o", str(exe)],
                   check=True, timeout=600)
    d = tmp_path / "files"
    d.mkdir()
    r = subprocess.run([str(exe), str(d)], capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "sanitize host ok" in r.stdout and "runtime error" not in r.stderr
