import os
import sys

# the library replays hipGraphs on the rig-latency path only with the HIP
# runtime's graph packet capture off (set before HIP initialises)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libmantis_amd.so")


@pytest.fixture(scope="session")
def landmark_map():
    from mantis_amd import synth

    return synth.load_map()
