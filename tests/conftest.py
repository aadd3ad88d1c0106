import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU; run via gpurun")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this container (run with gpurun)")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def control(tmp_path, monkeypatch):
    """Fresh control plane: config rooted in tmp_path, file-backed SQLite store, a SimFarm of 3 hosts
    (m1 CPU-only control node, w1/w2 with 8x MI355X each) registered as hosts."""
    monkeypatch.setenv("KOP_PBKDF2_ITERS", "1000")
    from kubeoperator_amd.control.conf import Config, set_config
    from kubeoperator_amd.control.domain import context
    from kubeoperator_amd.control.engine.simfarm import SimFarm
    from kubeoperator_amd.control.store import db

    cfg = Config(path=None)
    cfg["DATA_DIR"] = str(tmp_path / "data")
    set_config(cfg)
    db.reset_for_tests(cfg.db_url)
    db.init_db()
    farm = SimFarm(gpu_hosts={"10.0.0.2", "10.0.0.3"})
    context.set_transport_factory(lambda: farm)

    class CP:
        pass

    cp = CP()
    cp.cfg, cp.farm, cp.tmp = cfg, farm, tmp_path
    yield cp
    context.set_transport_factory(None)
