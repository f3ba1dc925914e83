"""A/B of the narrow-conv forms inside the bf16 step parity test: runs tests/test_step_bf16_gpu.py with tuning slot
16 set to each value in argv (0 direct, 1 none, 2 no forward, 3 no data gradient, 4 no weight gradient)."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]
from moegan_mi import _lib as L  # noqa: E402

rc = 0
for v in sys.argv[1:]:
    L.call("mg_set_tuning", 16, int(v))
    print(f"==== narrow tuning {v}", flush=True)
    sel = os.environ.get("SEL", "tests/test_step_bf16_gpu.py::test_bf16_c2_step_vs_oracle[8]").split()
    rc |= pytest.main(["-q", "-x", "-s", "--timeout", "300", "--timeout-method", "thread"] + sel)
sys.exit(rc)
