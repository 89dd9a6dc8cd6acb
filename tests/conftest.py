import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "aihab-clip_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the C-ABI kernels")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    import json
    import numpy as np

    cache = {}

    def get(tag):
        if tag not in cache:
            z = np.load(os.path.join(GOLDEN, f"{tag}.npz"))
            d = {k: z[k] for k in z.files}
            d["meta"] = json.loads(bytes(d["meta"]).decode())
            cache[tag] = d
        return cache[tag]
    return get
