"""Host-code sanitizers (SURVEY §5 race detection / sanitizers): the CPU image runtime
(csrc/cpu/imgproc.cpp) built with ASan + UBSan (incl. float-cast-overflow) and driven through every
exported function on odd / degenerate shapes and non-finite coordinates."""
import shutil

import pytest


@pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++')
def test_imgproc_asan_ubsan():
    from pytorch_raft_amd.build import build_sanitized
    exe, out = build_sanitized(run=True)
    assert 'imgproc sanitize: ok' in out, out
