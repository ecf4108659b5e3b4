"""CPU sanitizer leg: the host-side C this repo ships or tests
with -- the oracle's restatement, the reference's own fft2d transforms with
the restated glue (where /root/reference exists), the library's
context-free host entries (dcte_host.cpp), the plug-in glue and the fake
liblqr driving it -- built with -fsanitize=address,undefined and run by one
driver (tests/asan/asan_cpu.c).  Any sanitizer report aborts the driver;
every comparison it makes must hold.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "tests", "asan")


def _sanitizers_available():
    cc = shutil.which("gcc")
    if not cc:
        return False
    r = subprocess.run([cc, "-fsanitize=address,undefined", "-x", "c", "-", "-o", os.devnull],
                       input="int main(void){return 0;}", capture_output=True, text=True)
    return r.returncode == 0


@pytest.mark.skipif(not _sanitizers_available(), reason="gcc without ASan/UBSan runtimes")
def test_host_code_under_asan_and_ubsan():
    import dctenergy
    dctenergy.lib()                                   # the product library the plug-in links
    if os.path.isdir("/root/reference/src/fft2d"):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref-asan"], check=True)
    subprocess.run(["make", "-s", "-C", ASAN], check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([os.path.join(ASAN, "build", "asan_cpu")], capture_output=True, text=True,
                       env=env, timeout=900)
    print(r.stdout[-2000:], r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "asan_cpu: ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
