"""The text file reader of the device ingest (csrc/text_ring.h, bound as TextFileRing): the pread
reader into caller slots and the mapped reader (chunks handed out as pointers into the file's
mapping, which the GPU path page-locks so the copy engine reads the page cache directly).

Both must cut [lo, hi) into newline-aligned chunks of at most `chunk` bytes, in order, with the
line count of every chunk (a last line without a newline counts). Checked against the file bytes.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from mxstream.ops.native import load


def _file(tmp_path, n_lines, tail_newline=True, seed=0):
    rng = np.random.default_rng(seed)
    lines = [b"2019-08-28T10:%02d:00 www.channel%04d.com %d" % (i % 60, rng.integers(0, 999),
                                                              rng.integers(0, 10**8))
             for i in range(n_lines)]
    data = b"\n".join(lines) + (b"\n" if tail_newline else b"")
    p = tmp_path / "in.txt"
    p.write_bytes(data)
    return str(p), data


def _drain(ring, slots=None):
    out, got = [], 0
    ring.start()
    while True:
        slot, nbytes, nlines, end, eof, ptr = ring.next(2000)
        if slot < 0:
            assert eof
            break
        if ptr:
            b = ctypes.string_at(ptr, nbytes)
        else:
            b = slots[slot][:nbytes].numpy().tobytes()
        out.append((b, nlines, end))
        ring.release(slot)
        got += 1
    ring.close()
    return out


def _check(chunks, data, lo, hi, chunk):
    assert b"".join(c[0] for c in chunks) == data[lo:hi]
    pos = lo
    for b, nlines, end in chunks:
        assert 0 < len(b) <= chunk
        pos += len(b)
        assert end == pos - lo
        assert nlines == b.count(b"\n") + (0 if b.endswith(b"\n") else 1)
        if pos < hi:
            assert b.endswith(b"\n")  # newline-aligned cut


@pytest.mark.parametrize("tail_newline", [True, False])
@pytest.mark.parametrize("mapped", [False, True])
def test_text_ring_chunks_equal_file(tmp_path, mapped, tail_newline):
    path, data = _file(tmp_path, 60_000, tail_newline)
    m = load()
    chunk = 1 << 16
    for lo, hi in ((0, len(data)), (data.index(b"\n", 1000) + 1, len(data) - 5000)):
        if hi < len(data):
            hi = data.index(b"\n", hi) + 1
        if mapped:
            ring = m.TextFileRing.mapped(path, lo, hi, 3, chunk, 4)
            assert ring.map_bytes == len(data) and ring.map_base != 0
            chunks = _drain(ring)
        else:
            slots = [torch.empty(chunk, dtype=torch.uint8) for _ in range(3)]
            ring = m.TextFileRing(path, lo, hi, [(t.data_ptr(), t.numel()) for t in slots], chunk,
                                  4)
            chunks = _drain(ring, slots)
        _check(chunks, data, lo, hi, chunk)


def test_mapped_ring_rejects_range_past_eof(tmp_path):
    path, data = _file(tmp_path, 100)
    with pytest.raises(ValueError, match="past the end"):
        load().TextFileRing.mapped(path, 0, len(data) + 1, 3, 1 << 16, 2)


def test_mapped_ring_line_longer_than_chunk(tmp_path):
    p = tmp_path / "long.txt"
    p.write_bytes(b"x" * 5000 + b"\n" + b"y\n")
    ring = load().TextFileRing.mapped(str(p), 0, os.path.getsize(p), 3, 4096, 2)
    ring.start()
    with pytest.raises(RuntimeError, match="longer than the ingest chunk"):
        while True:
            slot, *_ = ring.next(2000)
            if slot < 0:
                break
            ring.release(slot)
    ring.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mapped", ["1", "seg", "0"])
def test_gpu_text_source_device_batches_equal_file(tmp_path, monkeypatch, mapped):
    """TextFileSource's device ingest (ring + copy stream) hands over device batches whose bytes
    are the file's, through the page-locked mapping (MXS_TEXT_MMAP=1; "seg": 1 MB segments, so
    chunks are copied in two pieces across segment boundaries) or pinned slots (0)."""
    import mxstream.runtime.sources as S

    monkeypatch.setattr(S, "_TEXT_MMAP", mapped != "0")
    if mapped == "seg":
        monkeypatch.setattr(S, "_TEXT_SEG", 1 << 20)
    path, data = _file(tmp_path, 200_000)
    src = S.TextFileSource(path, batch_size=1 << 14)
    src.columnar, src.ring, src.ring_device = True, True, "cuda"
    src.open(0, 1, None)
    assert src._mapped == (mapped != "0")
    got, lines = [], 0
    done = False
    while not done:
        out, done = src.poll(0)
        for tb in out:
            tb.ready.synchronize()
            got.append(tb.data.cpu().numpy().tobytes())
            lines += tb.n
    src.close()
    assert b"".join(got) == data
    assert lines == data.count(b"\n")
