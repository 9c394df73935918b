"""Device-scope stream-order events (acme_event_*, OrderEvent): a consumer stream
continues only after the producer stream's work before the record, as with torch's
events."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _slow_fill(x, value, s):
    # Enough queued work on s that an unordered reader would see the old contents.
    with torch.cuda.stream(s):
        a = torch.randn(2048, 2048, device=x.device)
        for _ in range(20):
            a = torch.tanh(a @ a * 1e-3)
        x.fill_(value)
        x.add_(a[0, 0] * 0)


def test_consumer_stream_sees_producer_writes():
    from acme_amd._lib import OrderEvent
    dev = torch.device("cuda:0")
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ev = OrderEvent()
    x = torch.zeros(1 << 20, device=dev)
    outs = []
    for it in range(1, 6):
        _slow_fill(x, float(it), s1)
        ev.record(s1)
        s2.wait_event(ev)  # torch calls ev.wait(s2)
        with torch.cuda.stream(s2):
            outs.append(x.clone())
        # the producer's next fill must not overwrite before the copy: order back
        s1.wait_stream(s2)
    torch.cuda.synchronize()
    for it, o in enumerate(outs, 1):
        assert torch.all(o == float(it)), it
    assert ev.query()
