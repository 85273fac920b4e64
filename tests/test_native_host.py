"""Host-code sanitizers: the native input-pipeline core (csrc/host/io_core.h) built
standalone under AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer, then
run: TFRecord round trip, Example decoding with a truncation / mutation fuzz pass, threaded
batch normalisation (csrc/host/selftest/io_selftest.cpp). GPU sanitizers are not available on
this pool, so sanitizers cover host code only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "host", "selftest", "io_selftest.cpp")


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_host_io_core_under_sanitizers(tmp_path, san):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "io_selftest")
    flags = ["-fsanitize=" + san, "-fno-omit-frame-pointer"]
    if "undefined" in san:
        flags.append("-fno-sanitize-recover=undefined")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-msse4.2", "-pthread", *flags, SRC, "-o", exe],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "io_selftest ok" in r.stdout
