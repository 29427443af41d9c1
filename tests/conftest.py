import faulthandler
import os
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# pytest's own faulthandler plugin is off (pytest.ini): its all-thread dump plus the extension
# module list pushed the failing test's name and the runtime's message out of a driver log's tail.
# Fatal-signal stacks go to a file instead, and every test announces itself on stderr first.
_FAULT_LOG = os.path.join(tempfile.gettempdir(), f"rdeic_pytest_faults_{os.getpid()}.log")
_fault_file = open(_FAULT_LOG, "w")
faulthandler.enable(file=_fault_file, all_threads=False)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librdeic_hip.so on the device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_runtest_logstart(nodeid, location):
    sys.stderr.write(f"\n[rdeic] start {nodeid} (fatal-signal stacks: {_FAULT_LOG})\n")
    sys.stderr.flush()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rdeic_amd import _lib
    _lib.load()
    return torch.device("cuda")
