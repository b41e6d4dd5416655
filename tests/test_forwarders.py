"""The reference-side forwarders (integration/*.cc): every ORBmatcher search,
Optimizer::LocalBundleAdjustment, the KeyFrameDatabase methods and the Frame
forwarders, compiled against test stand-ins of the reference headers
(tests/cxx/orbslam_mock) and run on two copies of a synthetic map -- one
through the forwarder, one through a CPU restatement of the reference method
(tests/cxx/forwarders_test.cpp).  Also checks that the code blocks
INTEGRATION.md quotes from integration/ are the compiled text."""
import re
import subprocess
from pathlib import Path

import pytest

from cxx_build import build_forwarders_test

ROOT = Path(__file__).resolve().parents[1]
N_CASES = 62   # 31 per seed, two seeds


def _run(exe):
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    ok = [l for l in r.stdout.splitlines() if re.search(r" ok \(", l)]
    assert r.returncode == 0 and "PASS: 0 mismatching" in r.stdout, r.stdout + r.stderr
    assert len(ok) == N_CASES, r.stdout
    return r.stdout


def test_forwarders_on_the_oracle():
    """The forwarders' own work (rows, flags, result application, map edits in
    order) with the oracle answering the orbx_* calls: no GPU needed."""
    _run(build_forwarders_test("oracle"))


def test_forwarders_link_against_liborbx():
    """The same sources link against the product library (the GPU test runs it)."""
    assert build_forwarders_test("liborbx").exists()


@pytest.mark.gpu
def test_forwarders_on_the_gpu():
    """Every forwarder on the device, against the restated reference on the CPU."""
    out = _run(build_forwarders_test("liborbx"))
    print(out)


def test_integration_md_quotes_compiled_sources():
    """Each ```cpp block preceded by <!-- from FILE --> is a verbatim slice of FILE."""
    text = (ROOT / "INTEGRATION.md").read_text()
    blocks = re.findall(r"<!-- from (\S+) -->\n```cpp\n(.*?)```", text, re.S)
    assert len(blocks) >= 8, "INTEGRATION.md lost its quoted forwarders"
    for path, body in blocks:
        src = (ROOT / path).read_text()
        assert body in src, f"INTEGRATION.md block from {path} differs from the source:\n{body[:200]}"
