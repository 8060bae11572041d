"""Text ingestion on the GPU: delimited lines -> typed columns.

``parse_text_gpu`` uploads a batch of text once, finds the line starts (order-preserving
wave-ballot / tile-scan / write kernels over the bytes, csrc/kernels_hip.hip `line_starts`), and runs the gfx950 ``parse_text`` kernel (csrc/parse_hip.hip): one thread per
line, Java field semantics shared with the host runtime. Lines the kernel flags (inputs outside
its exact fast paths, or real errors) are re-parsed by the C++ runtime on the host and patched
into the device columns, so results are bit-identical to ``parse_lines`` on the CPU; a genuine
parse error raises the same Java exception text.

Field kinds (``FK_*``) are those of csrc/runtime.cpp. String fields produce a 64-bit FNV-1a key
(``int64``) plus the Java ``String.hashCode`` (``int32``, for key groups) instead of dictionary ids.
"""
from __future__ import annotations

import numpy as np
import torch

from .native import load

FK_STR, FK_DOUBLE, FK_LONG, FK_TS_INTSEC, FK_TS_MS, FK_INT, FK_RAW_LONG = range(7)

_FNV_OFF, _FNV_PRIME, _M64 = 0xcbf29ce484222325, 0x100000001b3, (1 << 64) - 1


class ParseError(ValueError):
    pass


def fnv1a64(b: bytes) -> int:
    h = _FNV_OFF
    for c in b:
        h = ((h ^ c) * _FNV_PRIME) & _M64
    if h in (_M64, _M64 - 1):  # -1 / -2 are the tables' reserved keys
        h -= 2
    return h - (1 << 64) if h >= 1 << 63 else h


def pinned_text_batch(data: bytes) -> torch.Tensor:
    """Stage a text batch in page-locked host memory, as the socket reader's ring slots are
    (SURVEY.md F-src): ``parse_text_gpu`` then uploads it with one DMA instead of a pageable
    copy through the driver's bounce buffer."""
    t = torch.empty(len(data), dtype=torch.uint8, pin_memory=torch.cuda.is_available())
    if len(data):
        t.numpy()[:] = np.frombuffer(data, dtype=np.uint8)
    return t


def parse_text_gpu(data, spec: list[tuple[int, int]], sep: str = " ", offset_s: int = 0,
                   device="cuda", *, ready=None, min_line_bytes: int = 8) -> list:
    """Returns one entry per spec field: a float64/int64 device tensor, or for FK_STR a
    (key int64, java_hash int32) pair of device tensors.

    ``data`` is ``bytes`` or a 1-D uint8 tensor (a pinned host batch from ``pinned_text_batch``,
    uploaded asynchronously, or a batch already on the device -- ``ready``: an event after which
    its copy, e.g. on a side stream, is complete).

    No host pass over the text: the line-start index is sized for ``n_bytes / min_line_bytes``
    lines (line_starts writes at most that many, counts them all), the parse kernel reads the
    device line count, and ONE readback returns (lines, flagged lines). A batch with more lines
    than the bound -- shorter lines than assumed -- is redone with the exact size."""
    if not spec or len(spec) > 8:
        raise ValueError("1..8 fields")
    dev = torch.device(device)
    m = load()
    st = torch.cuda.current_stream(dev).cuda_stream
    if isinstance(data, torch.Tensor):
        if data.dtype != torch.uint8 or data.dim() != 1:
            raise ValueError("text batch tensor must be 1-D uint8")
        n_bytes = data.numel()
        if ready is not None:
            torch.cuda.current_stream(dev).wait_event(ready)
        buf = (data.to(dev, non_blocking=data.is_pinned()) if n_bytes
               else torch.zeros(1, dtype=torch.uint8, device=dev))
        host = data
    else:
        raw = np.frombuffer(data, dtype=np.uint8)
        n_bytes = raw.size
        buf = torch.from_numpy(raw.copy()).to(dev) if n_bytes else torch.zeros(
            1, dtype=torch.uint8, device=dev)
        host = None
    nf = len(spec)
    if n_bytes == 0:
        return [torch.empty(0, dtype=torch.float64 if k == FK_DOUBLE else torch.int64, device=dev)
                if k != FK_STR else (torch.empty(0, dtype=torch.int64, device=dev),
                                     torch.empty(0, dtype=torch.int32, device=dev))
                for _, k in spec]
    scratch = torch.empty(max(1, m.gpu_filter_compact_scratch_bytes(n_bytes)), dtype=torch.uint8,
                          device=dev)
    ctl = torch.zeros(2, dtype=torch.int64, device=dev)  # [0] lines  [1] flagged lines (u32)
    bound = min(n_bytes, n_bytes // max(1, int(min_line_bytes)) + 256)
    while True:
        starts_buf = torch.empty(max(bound, 1), dtype=torch.int64, device=dev)
        cols = torch.empty(nf * bound, dtype=torch.int64, device=dev)
        jh = torch.zeros(nf * bound, dtype=torch.int32, device=dev)
        status = torch.empty(bound, dtype=torch.uint8, device=dev)
        ctl.zero_()
        m.gpu_line_starts(buf.data_ptr(), n_bytes, scratch.data_ptr(), starts_buf.data_ptr(),
                          ctl[0:1].data_ptr(), st, bound)
        m.gpu_parse_text(buf.data_ptr(), n_bytes, starts_buf.data_ptr(), bound,
                         [f for f, _ in spec], [k for _, k in spec], sep, int(offset_s),
                         cols.data_ptr(), jh.data_ptr(), status.data_ptr(), st,
                         nlines_dev=ctl[0:1].data_ptr(), nflag=ctl[1:2].data_ptr())
        n, nflag = ctl.tolist()  # the batch's one host synchronisation
        nflag &= 0xFFFFFFFF
        if n <= bound:
            break
        bound = n  # lines shorter than min_line_bytes: exact size, once
    starts = starts_buf[:n]
    if nflag:
        bad = torch.nonzero(status[:n]).flatten()
        if host is not None:
            data = host.cpu().numpy().tobytes()
        # the kernel laid columns out with the device count n as the column stride
        _host_patch(m, data, starts.cpu().numpy(), bad.cpu().numpy(), spec, sep, offset_s,
                    cols, jh, n)
    out = []
    for f, (_, kind) in enumerate(spec):
        c = cols[f * n:(f + 1) * n]
        if kind == FK_DOUBLE:
            out.append(c.view(torch.float64))
        elif kind == FK_STR:
            out.append((c, jh[f * n:(f + 1) * n]))
        else:
            out.append(c)
    return out


def _host_patch(m, data: bytes, starts: np.ndarray, bad: np.ndarray, spec, sep, offset_s,
                cols: torch.Tensor, jh: torch.Tensor, n: int) -> None:
    """Re-parse flagged lines with the C++ runtime (exact Java semantics / exception text)."""
    ends = np.append(starts[1:] - 1, len(data))
    lines = []
    for i in bad.tolist():
        line = data[starts[i]:ends[i]]
        if line.endswith(b"\r"):
            line = line[:-1]
        lines.append(line)
    d = m.StringDict()
    host_spec = [(f, k) for f, k in spec]
    res_cols, nparsed, err_idx, err = m.parse_lines(b"\n".join(lines) + b"\n", host_spec, sep, d,
                                                    int(offset_s))
    if err:
        raise ParseError(f"line {int(bad[err_idx]) + 1}: {err}")
    dev = cols.device
    idx = torch.from_numpy(bad.astype(np.int64)).to(dev)
    strings = d.strings()
    for f, (_, kind) in enumerate(spec):
        vals = res_cols[f]
        if kind == FK_STR:
            keys = np.array([fnv1a64(strings[i].encode()) for i in vals.tolist()], dtype=np.int64)
            hs = np.array([m.java_string_hash(strings[i]) for i in vals.tolist()], dtype=np.int32)
            jh[f * n + idx] = torch.from_numpy(hs).to(dev)
            vals = keys
        elif kind == FK_DOUBLE:
            vals = np.asarray(vals, dtype=np.float64).view(np.int64)
        cols[f * n + idx] = torch.from_numpy(np.ascontiguousarray(vals, dtype=np.int64)).to(dev)
