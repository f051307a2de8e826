"""bench.py's transport fallback order (host logic only, no GPU): the requested decoder
mode first, then RCCL -> IPC -> replicas for N > 1, one GPU for N = 1."""
import bench


def test_multi_gpu_default_falls_back_rccl_ipc_replicas():
    assert bench.transport_candidates(8, False, "rccl", False) == ["tp-rccl", "tp-ipc", "replica"]


def test_multi_gpu_ipc_requested():
    assert bench.transport_candidates(2, False, "ipc", False) == ["tp-ipc", "replica"]


def test_multi_gpu_replicas_requested():
    assert bench.transport_candidates(4, False, "rccl", True) == ["replica"]


def test_one_gpu():
    assert bench.transport_candidates(1, False, "rccl", False) == ["single"]
    assert bench.transport_candidates(1, True, "ipc", False) == ["tp-ipc", "single"]
    assert bench.transport_candidates(1, True, "rccl", False) == ["tp-rccl", "single"]
