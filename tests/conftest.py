import asyncio
import inspect
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs the MI355X box (run by the driver's `pytest -m gpu` tier)")
    config.addinivalue_line("markers", "slow: multi-second scale / soak tests")


@pytest.hookimpl(tryfirst=True)
def pytest_pyfunc_call(pyfuncitem):
    """Run `async def` tests on a fresh event loop (no pytest-asyncio in this image)."""
    fn = pyfuncitem.obj
    if inspect.iscoroutinefunction(fn):
        sig = inspect.signature(fn)
        kwargs = {k: v for k, v in pyfuncitem.funcargs.items() if k in sig.parameters}
        asyncio.run(asyncio.wait_for(fn(**kwargs), timeout=float(os.environ.get("NCC_TEST_TIMEOUT", "120"))))
        return True
    return None
