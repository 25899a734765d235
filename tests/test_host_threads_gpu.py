"""The JW_HOST path driven from 8 C threads at once on one shared plan (tests/c/host_threads.c,
MODWTThreadSafetyTest.java:23-104 pattern: DIRECT and AUTO calls, with jw_release_caches()
racing them as clearFilterCache() does there), every result bit-exact against the oracle --
once on the calling thread's default device and once with every thread selecting device 0
explicitly (jw_set_device)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

BIN = os.path.join(os.path.dirname(__file__), "c", "host_threads")


@pytest.mark.parametrize("device", [None, 0])
def test_host_path_eight_threads_bit_exact(device):
    assert os.path.exists(BIN), "tests/c/host_threads is built by __graft_entry__.build()"
    r = subprocess.run([BIN] + ([] if device is None else [str(device)]), capture_output=True,
                       text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
