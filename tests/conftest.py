"""Test configuration.

Paths: the drop-in modules live in ``sdp-net_amd/`` (imported as top-level
``model`` / ``layers`` / ...), the CPU oracle in ``oracle/`` (test
infrastructure), the golden fixtures and the portable weight generator in
``tests/golden/``.  Nothing here reads /root/reference.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("sdp-net_amd", "oracle", os.path.join("tests", "golden")):
    p = os.path.join(REPO, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
