"""The HIP runtime's one-call stream helpers (hip/runtime/hip_runtime.cpp: event_create /
event_record / stream_wait_event / event_synchronize / event_elapsed_ms / memcpy_async /
memset_async), which the resident batch verify issues its pipeline with: ordering across two
streams, both copy directions, and the refusal of an unknown direction."""
import pytest

pytestmark = pytest.mark.gpu


def test_stream_helpers_order_copies_across_streams(gpu):
    import numpy as np
    import torch

    from nodexa_chain_core_amd.ops import runtime

    h = runtime.hip()
    n = 1 << 20
    src = torch.arange(n, dtype=torch.int32).pin_memory()
    dev = torch.empty(n, dtype=torch.int32, device="cuda")
    back = torch.zeros(n, dtype=torch.int32).pin_memory()
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    sa, sb = int(a.cuda_stream), int(b.cuda_stream)
    t0, t1, ready = h.event_create(True), h.event_create(True), h.event_create()
    try:
        h.event_record(t0, sa)
        h.memcpy_async(dev.data_ptr(), src.data_ptr(), n * 4, sa, "htod")
        h.memset_async(dev.data_ptr() + 4 * 16, 0, 4 * 16, sa)  # elements 16..31 zeroed after the upload
        h.event_record(ready, sa)
        h.stream_wait_event(sb, ready)  # the download on the other stream waits for both
        h.memcpy_async(back.data_ptr(), dev.data_ptr(), n * 4, sb, "dtoh")
        h.event_record(t1, sb)
        h.event_synchronize(t1)
        want = np.arange(n, dtype=np.int32)
        want[16:32] = 0
        assert np.array_equal(back.numpy(), want)
        assert h.event_elapsed_ms(t0, t1) > 0
        with pytest.raises(ValueError):
            h.memcpy_async(back.data_ptr(), dev.data_ptr(), 4, sb, "sideways")
    finally:
        for e in (t0, t1, ready):
            h.event_destroy(e)
