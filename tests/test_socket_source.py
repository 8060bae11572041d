"""socketTextStream (SocketTextStreamFunction semantics, every reference job's source,
Main.java:17): a local TCP server plays `nc -lk 8080` (chapter1/README.md:66-68). The columnar
path reads raw batches; with several ranks the socket is read on rank 0 and its batches are
spread over every rank (K18, the p=1 source -> p=N rebalance of Main.java:17 -> 18)."""
import socket
import threading
from collections import Counter

import pytest

from test_datastream_device_exchange import _lines


def _serve(payload: bytes):
    srv = socket.socket()
    srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]

    def run():
        conn, _ = srv.accept()
        for i in range(0, len(payload), 4096):  # arrives in pieces, like a typing user / nc
            conn.sendall(payload[i:i + 4096])
        conn.close()
        srv.close()

    th = threading.Thread(target=run, daemon=True)
    th.start()
    return port, th


def _job_socket(port, comm=None, ingest="device"):
    from mxstream.api.environment import StreamExecutionEnvironment
    from mxstream.models import chapters as C

    out = []
    env = StreamExecutionEnvironment(4).set_output(out.append)
    env.config.text_ingest = ingest
    env._comm = comm
    C.build_bandwidth_event_time(env, env.socket_text_stream("127.0.0.1", port))
    env.execute("bw-socket")
    return out


def _job_collection(lines):
    from mxstream.api.environment import StreamExecutionEnvironment
    from mxstream.models import chapters as C

    out = []
    env = StreamExecutionEnvironment(4).set_output(out.append)
    C.build_bandwidth_event_time(env, env.from_collection(lines))
    env.execute("bw-collection")
    return out


@pytest.mark.parametrize("ingest", ["host", "device"])
def test_socket_job_equals_collection(ingest):
    lines = _lines(1500, 19)
    ref = _job_collection(lines)
    assert ref
    port, th = _serve(("\r\n".join(lines) + "\n").encode())  # '\r' is stripped (Flink)
    got = _job_socket(port, ingest=ingest)
    th.join(timeout=30)
    assert Counter(got) == Counter(ref)


@pytest.mark.parametrize("world", [2, 3])
def test_socket_batches_spread_over_ranks(world):
    from mxstream.parallel.comm import run_loopback
    from mxstream.runtime import sources as S

    lines = _lines(1500, 19)
    ref = _job_collection(lines)
    port, th = _serve(("\n".join(lines) + "\n").encode())
    seen = Counter()
    orig = S.SocketTextSource._poll_spread

    def spy(self):
        items, eof = orig(self)
        seen[self.comm.rank] += sum(it.n for it in items)
        return items, eof

    S.SocketTextSource._poll_spread = spy
    try:
        res = run_loopback(world, lambda comm: _job_socket(port, comm))
    finally:
        S.SocketTextSource._poll_spread = orig
    th.join(timeout=30)
    got = [l for out in res for l in out]
    assert Counter(got) == Counter(ref)
    assert sum(seen.values()) == len(lines) and all(seen[r] > 0 for r in range(world))


def test_socket_reader_back_pressure():
    """The reader queue is bounded: with a slow consumer the reader thread waits for space
    (TCP flow control then slows the sender) and no line is lost."""
    import time

    from mxstream.ops.native import load

    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]
    n = 50_000

    def serve():
        c, _ = srv.accept()
        c.sendall(b"".join(b"%d\n" % i for i in range(n)))
        c.close()
        srv.close()

    th = threading.Thread(target=serve)
    th.start()
    r = load().SocketSource("127.0.0.1", port, "\n", 0, max_queue=256)
    r.start()
    got = []
    while True:
        data, k, eof, err = r.poll(100, 100)
        assert not err
        got += data.decode().split("\n")[:k]
        if eof:
            break
        time.sleep(0.0005)
    th.join()
    r.close()
    assert got == [str(i) for i in range(n)]
    assert r.blocked() > 0
