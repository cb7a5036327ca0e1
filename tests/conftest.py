import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import helpers  # noqa: E402,F401  (sets sys.path for the package and the oracle)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libcrdtgpu.so on the device)")


# Run order for `pytest -m gpu -x`: the reference tests (config 1) and the per-config
# oracle-parity tests of the hot path first, so a failure or stall in a peripheral
# test can never leave a config unreached; then everything else in file order; the
# probes and the test that spawns two GPU processes last.
_FIRST = (
    "test_scenarios_gpu.py::",
    "test_gpu_parity.py::test_golden_merges_on_gpu",
    "test_gpu_parity.py::test_config2_full_size",
    "test_gpu_parity.py::test_exchange_config2_full_size",
    "test_gpu_parity.py::test_config3_full_size",
    "test_gpu_parity.py::test_gen_replicas_and_config5_fold",
    "test_gpu_parity.py::test_config5_bench_size",
    "test_gpu_tiles.py::test_config4_full_size_exchange",
    "test_gpu_parity.py::test_config4_zipf_slice_exact",
)
_LAST = (
    "test_gpu_probe.py::",
    "test_gpu_comm.py::",
    "test_gpu_multirank.py::",
)


def _rank(item):
    nid = item.nodeid.split("/")[-1]
    for i, p in enumerate(_FIRST):
        if nid.startswith(p):
            return (0, i)
    for i, p in enumerate(_LAST):
        if nid.startswith(p):
            return (2, i)
    return (1, 0)


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=_rank)  # stable: file order kept inside each group
