"""Device-scope stream ordering (rs_event_*, _lib.DeviceEvent): an event created with
hipEventDisableSystemFence orders two streams of one device exactly as a torch event does —
the waiting stream sees everything the recording stream queued before the record."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_device_event_orders_two_streams():
    from recommender_amd import _lib as L

    L.load()
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    n = 1 << 24
    x = torch.empty(n, device="cuda")
    ev = L.DeviceEvent()
    for k in range(3):  # the event re-recorded each round (as the optimizer's persistent events)
        with torch.cuda.stream(a):
            x.fill_(float(k + 1))
            y = x * 2.0
        ev.record(a)
        ev.wait_by(b)
        with torch.cuda.stream(b):
            z = y.sum()
        y.record_stream(b)
        torch.cuda.synchronize()
        assert z.item() == 2.0 * (k + 1) * n


def test_stream_wait_stream_and_record_event_helpers():
    from recommender_amd import _lib as L

    L.load()
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    x = torch.empty(1 << 22, device="cuda")
    with torch.cuda.stream(a):
        x.fill_(3.0)
    L.stream_wait_stream(b, a)
    with torch.cuda.stream(b):
        s1 = x.sum()
    e = L.record_event(a)
    assert isinstance(e, L.DeviceEvent) == L.DEVICE_EVENTS
    L.stream_wait_event(b, e)
    torch.cuda.synchronize()
    assert s1.item() == 3.0 * (1 << 22)
