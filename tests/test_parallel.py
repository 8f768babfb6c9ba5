

def test_transport_check_by_device_identity():
    import pytest

    """``rccl`` with two ranks on one device is refused with the fix named;
    ``ipc`` accepts shared devices; distinct devices pass."""
    from omnia_amd.parallel.state import check_transport

    check_transport("rccl", [("h", "gpu0"), ("h", "gpu1"), ("h2", "gpu0")])
    check_transport("ipc", [("h", "gpu0"), ("h", "gpu0")])
    with pytest.raises(RuntimeError, match="OMNIA_TP_TRANSPORT=ipc"):
        check_transport("rccl", [("h", "gpu0"), ("h", "gpu1"), ("h", "gpu0")])
