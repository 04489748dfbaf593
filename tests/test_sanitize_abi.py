"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer run over the HIP library's whole C ABI (CPU, no GPU).

``pathnet_gym_amd/_sanitize.py`` compiles every ``csrc/*.hip`` with the sanitizers on the host half only
(``-Xarch_host -fsanitize=...``) and links a generated harness that calls each exported function from the ctypes
table under six argument scenarios (zeros, one, typical, odd, -1, 4096).  Launches fail with hipErrorNoDevice
here; everything before them -- argument validation, grid / LDS-size arithmetic, shape dispatch, host helpers --
runs under the sanitizers.  The first build takes ~2 minutes (content-hash cached afterwards).
"""
import os
import shutil

import pytest

from pathnet_gym_amd import _build


@pytest.mark.skipif(not (os.path.exists(_build.HIPCC) and os.path.exists("/opt/rocm/lib/llvm/bin/clang++")),
                    reason="needs hipcc / clang++ from ROCm")
def test_c_abi_is_clean_under_asan_and_ubsan():
    from pathnet_gym_amd import _sanitize
    from pathnet_gym_amd.ops import _lib
    _sanitize.build()
    r = _sanitize.run(timeout=600)
    out = r.stdout + r.stderr
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    n_fn = sum(1 for k in _lib._SIGS if not k.startswith("fast_conv_set_"))
    assert f"abi harness: {n_fn * len(_sanitize.SCENARIOS)} calls, no sanitizer report" in r.stdout
