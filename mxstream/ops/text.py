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
                   device="cuda") -> list:
    """Returns one entry per spec field: a float64/int64 device tensor, or for FK_STR a
    (key int64, java_hash int32) pair of device tensors.

    ``data`` is ``bytes`` or a 1-D uint8 tensor (a pinned host batch from ``pinned_text_batch``
    or a batch already on the device); a pinned batch is uploaded asynchronously."""
    if not spec or len(spec) > 8:
        raise ValueError("1..8 fields")
    dev = torch.device(device)
    m = load()
    if isinstance(data, torch.Tensor):
        if data.dtype != torch.uint8 or data.dim() != 1:
            raise ValueError("text batch tensor must be 1-D uint8")
        n_bytes = data.numel()
        buf = (data.to(dev, non_blocking=data.is_pinned()) if n_bytes
               else torch.zeros(1, dtype=torch.uint8, device=dev))
        host = data
    else:
        raw = np.frombuffer(data, dtype=np.uint8)
        n_bytes = raw.size
        buf = torch.from_numpy(raw.copy()).to(dev) if n_bytes else torch.zeros(
            1, dtype=torch.uint8, device=dev)
        host = None
    # Line starts (0 and every byte after a newline, below n_bytes: a trailing newline starts no
    # line) by the order-preserving ballot/scan/write kernels; one host sync for the count. The
    # index array is sized by the line count when the host holds the text (a device-only batch
    # falls back to the byte count, the only bound known without reading it).
    from .ingest import count_lines

    if host is not None and host.device.type == "cpu":
        bound = count_lines(host) + 1
    elif host is None:
        bound = count_lines(data) + 1
    else:
        bound = n_bytes
    starts_buf = torch.empty(max(min(bound + 64, n_bytes), 1), dtype=torch.int64, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    scratch = torch.empty(max(1, m.gpu_filter_compact_scratch_bytes(n_bytes)), dtype=torch.uint8,
                          device=dev)
    m.gpu_line_starts(buf.data_ptr(), n_bytes, scratch.data_ptr(), starts_buf.data_ptr(),
                      total.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    n = int(total.item()) if n_bytes else 0
    starts = starts_buf[:n]
    nf = len(spec)
    cols = torch.empty(nf * max(n, 1), dtype=torch.int64, device=dev)
    jh = torch.zeros(nf * max(n, 1), dtype=torch.int32, device=dev)
    status = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
    if n:
        m.gpu_parse_text(buf.data_ptr(), n_bytes, starts.contiguous().data_ptr(), n,
                         [f for f, _ in spec], [k for _, k in spec], sep, int(offset_s),
                         cols.data_ptr(), jh.data_ptr(), status.data_ptr(),
                         torch.cuda.current_stream(dev).cuda_stream)
        bad = torch.nonzero(status[:n]).flatten()
        if bad.numel():
            if host is not None:
                data = host.cpu().numpy().tobytes()
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
