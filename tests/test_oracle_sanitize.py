"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
§5 aux: "ASan/UBSan build of the oracle").  `make -C oracle sanitize`
builds oracle/sancheck.cpp with every oracle source; it drives the
monocular and stereo paths (both summation orders, keyframe insertion) and
the rig over a scene whose view drifts to the image border, so patches and
bilinear taps leave the level buffers — where the reference reads past its
cv::Mat (include/common.h:35-41) and starts from an uninitialised
frame_cnt (include/viso.h:38), the oracle's defined restatement must stay
clean.  Host-only (no GPU)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_oracle_clean_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", ORACLE, "sanitize"], check=True, timeout=600)
    # verify_asan_link_order=0: other preloaded libraries may precede the
    # ASan runtime in the process's library list
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ORACLE, "_build", "oracle_sancheck")], capture_output=True, text=True,
                       timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "sancheck ok" in r.stdout
    assert "runtime error" not in out and "AddressSanitizer" not in out and "LeakSanitizer" not in out
    # the drivers reached tracking (stereo) and the rig's tracking
    assert "stereo: state 1" in r.stdout and "rig: state 1" in r.stdout
