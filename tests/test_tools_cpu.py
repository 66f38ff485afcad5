"""Every measurement script under tools/ imports (the evidence runs on the GPU box depend on them;
a missing helper module must fail here, not there).  Importing runs no GPU code: each tool keeps
its work in main()."""
import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = sorted(f[:-3] for f in os.listdir(os.path.join(ROOT, "tools")) if f.endswith(".py"))


@pytest.mark.parametrize("name", TOOLS)
def test_tool_imports(name):
    sys.path.insert(0, ROOT)
    try:
        importlib.import_module(f"tools.{name}")
    finally:
        sys.path.remove(ROOT)
