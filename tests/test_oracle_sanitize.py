"""The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer (host only): `make -C oracle
sanitize` builds oracle/sanitize_main.c with the oracle sources (-fsanitize=address,undefined,
abort on the first report) and drives every public orc_* entry point -- tape and Philox resets,
caller actions / deltas / sampled actions, W = 1, 5, 10, 21, a mass-truncation run, a custom
obstacle config and the createBoard profile."""
import os
import shutil
import subprocess

import pytest

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None, reason="no host C compiler")
def test_oracle_asan_ubsan_clean():
    r = subprocess.run(["make", "-s", "-C", ORACLE, "sanitize"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitize: OK" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
