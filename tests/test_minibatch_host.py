"""
Host-side checks of the device minibatch order (oracle/minibatch.py, the restatement the GPU
rows kernel is checked against) and of DeviceDataLoader's argument handling: every epoch is a
permutation of the rows (as DataLoader(shuffle=True) visits each row once per epoch), batches
partition it, the order differs between epochs, and sequential order is the identity.
"""
import pytest
import torch

from mininf_amd import _native as nat
from mininf_amd.data import DeviceDataLoader
from oracle import minibatch as oracle


@pytest.mark.parametrize("n,batch", [(1000, 64), (37, 37), (4096, 512), (10, 3)])
def test_epochs_are_permutations(n, batch):
    batches = -(-n // batch)
    for epoch in range(3):
        rows = []
        for b in range(batches):
            count = min(batch, n - b * batch)
            rows += oracle.batch_rows(epoch * batches + b, n, batch, batches, True, 7, count)
        assert sorted(rows) == list(range(n))
    first = [oracle.batch_rows(b, n, batch, batches, True, 7, min(batch, n - b * batch))
             for b in range(batches)]
    second = [oracle.batch_rows(batches + b, n, batch, batches, True, 7,
                                min(batch, n - b * batch)) for b in range(batches)]
    if n > 10:
        assert first != second


def test_sequential_order_and_seeds():
    assert oracle.batch_rows(3, 100, 10, 10, False, 1, 10) == list(range(30, 40))
    a = oracle.batch_rows(0, 1000, 100, 10, True, 1, 100)
    b = oracle.batch_rows(0, 1000, 100, 10, True, 2, 100)
    assert a != b


def test_loader_rejects_host_tensors_and_mismatched_sizes():
    with pytest.raises(nat.NativeError):
        DeviceDataLoader(torch.zeros(10, 2), batch_size=2)
    with pytest.raises(ValueError, match="Size mismatch"):
        DeviceDataLoader(torch.zeros(10), torch.zeros(9), batch_size=2)
    with pytest.raises(ValueError, match="batch_size"):
        DeviceDataLoader(torch.zeros(10), batch_size=0)
