"""Loopback parameter-server plumbing (BASELINE.json config 1): the reference's
wire framing in front of DataStore.handlePush / handleFetch.

Framing (reference): every message is a big-endian int32 length followed by the
message (PSAgent.DataBuffer.readData, PSAgent.java:27-62); messages are
DataBusProtocol's (DataBusProtocol.java:17-22, 124-337): a BE int32 type, then
  PushRequest   DataDesc (6 BE int32, DataDesc.java:62-69), BE int32 length, the
                LE record bytes, BE int32 name length, name bytes;
  PushResponse  BE int32 success;
  FetchRequest  BE int32 name length, name, rows and cols KeyCollections
                (KeyCollection.java:34-69, KeyRange.java:43-66, KeyList.java:31-57);
  FetchResponse DataDesc, BE length, record bytes, BE name length, name;
  CloseRequest  nothing more.
PSServer mirrors PSAgent.run / handle (PSAgent.java:161-285): one selector
thread, a push applied synchronously under the store's lock and acknowledged
after the apply. PSClient is the worker side (Session / WorkerAgent), blocking.
The stores are anything with handlePush(format, bytes) / handleFetch(format,
rows): distml_amd.DataStore in production. This is plumbing for config 1 and
end-to-end tests; a JVM deployment keeps its own transport.
"""
from __future__ import annotations

import selectors
import socket
import struct
import threading
from typing import Dict, List, Optional, Tuple

from .datadesc import ALL, EMPTY, AllKeys, DataDesc, KeyCollection, KeyList, KeyRange

MSG_FETCH_REQUEST, MSG_FETCH_RESPONSE, MSG_PUSH_REQUEST, MSG_PUSH_RESPONSE, MSG_SYNC_REQUEST, MSG_CLOSE = range(6)


def _i32(x: int) -> bytes:
    return struct.pack(">i", x)


class _Reader:
    """AbstractDataReader over one message (big-endian, like DataInputStream)."""

    def __init__(self, buf: bytes):
        self.buf, self.pos = buf, 0

    def _take(self, fmt: str, n: int):
        if self.pos + n > len(self.buf):
            raise EOFError("truncated message")
        v = struct.unpack_from(fmt, self.buf, self.pos)[0]
        self.pos += n
        return v

    def i32(self) -> int:
        return self._take(">i", 4)

    def i64(self) -> int:
        return self._take(">q", 8)

    def raw(self, n: int) -> bytes:
        if n < 0 or self.pos + n > len(self.buf):
            raise EOFError("truncated message")
        v = self.buf[self.pos:self.pos + n]
        self.pos += n
        return v

    def desc(self) -> DataDesc:
        return DataDesc.read(self.raw(24))


def write_keys(keys: KeyCollection, fmt: DataDesc) -> bytes:
    """KeyCollection.write (KeyCollection.java:34-36, KeyRange.java:43-54, KeyList.java:31-43):
    keys are written as int or long by the matrix's key type."""
    kfmt = ">i" if fmt.keyType == DataDesc.KEY_TYPE_INT else ">q"
    if isinstance(keys, AllKeys):
        return _i32(KeyCollection.TYPE_ALL)
    if isinstance(keys, KeyRange):
        return _i32(KeyCollection.TYPE_RANGE) + struct.pack(kfmt, keys.firstKey) + struct.pack(kfmt, keys.lastKey)
    if isinstance(keys, KeyList):
        ks = list(keys)
        return _i32(KeyCollection.TYPE_LIST) + _i32(len(ks)) + b"".join(struct.pack(kfmt, k) for k in ks)
    return _i32(KeyCollection.TYPE_EMPTY)


def read_keys(r: _Reader, fmt: DataDesc) -> KeyCollection:
    """KeyCollection.readKeyCollection (KeyCollection.java:41-69)."""
    t = r.i32()
    get = r.i32 if fmt.keyType == DataDesc.KEY_TYPE_INT else r.i64
    if t == KeyCollection.TYPE_ALL:
        return ALL
    if t == KeyCollection.TYPE_EMPTY:
        return EMPTY
    if t == KeyCollection.TYPE_RANGE:
        first = get()
        return KeyRange(first, get())
    if t == KeyCollection.TYPE_LIST:
        return KeyList([get() for _ in range(r.i32())])
    raise ValueError("KeyHash collections are not served (SURVEY defect 2)")


def _name(name: str) -> bytes:
    b = name.encode()
    return _i32(len(b)) + b


def push_request(name: str, fmt: DataDesc, data: bytes) -> bytes:
    """DataBusProtocol.PushRequest.write (Data.write :148-154, :287-292)."""
    return _i32(MSG_PUSH_REQUEST) + fmt.write() + _i32(len(data)) + bytes(data) + _name(name)


def fetch_request(name: str, fmt: DataDesc, rows: KeyCollection, cols: KeyCollection = ALL) -> bytes:
    """DataBusProtocol.FetchRequest.write (:194-203)."""
    return _i32(MSG_FETCH_REQUEST) + _name(name) + write_keys(rows, fmt) + write_keys(cols, fmt)


def frame(msg: bytes) -> bytes:
    """The length prefix PSAgent.DataBuffer reads first (PSAgent.java:41-50)."""
    return _i32(len(msg)) + msg


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    out = bytearray()
    while len(out) < n:
        chunk = sock.recv(n - len(out))
        if not chunk:
            raise ConnectionError("peer closed")
        out += chunk
    return bytes(out)


def recv_frame(sock: socket.socket) -> bytes:
    n = struct.unpack(">i", _recv_exact(sock, 4))[0]
    if n < 0:
        raise ValueError("negative frame length")
    return _recv_exact(sock, n)


class PSServer:
    """One parameter-server shard: {matrix name: (store, format)} behind a
    selector loop on 127.0.0.1. `pushes` records (name, bytes) in the order the
    pushes were applied: the order that defines the reference's result."""

    def __init__(self, stores: Dict[str, Tuple[object, DataDesc]], host: str = "127.0.0.1", port: int = 0):
        self.stores = stores
        self.locks = {name: threading.Lock() for name in stores}
        self.pushes: List[Tuple[str, bytes]] = []
        self.errors: List[BaseException] = []
        self._ss = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._ss.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._ss.bind((host, port))
        self._ss.listen(16)
        self._ss.setblocking(False)
        self.address = self._ss.getsockname()
        self._sel = selectors.DefaultSelector()
        self._sel.register(self._ss, selectors.EVENT_READ)
        self._conns: List[socket.socket] = []
        self._running = False
        self._thread: Optional[threading.Thread] = None

    def start(self) -> "PSServer":
        self._running = True
        self._thread = threading.Thread(target=self._run, name="PSAgent", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._running = False
        if self._thread:
            self._thread.join(timeout=10)
        for c in list(self._conns):
            self._drop(c)
        self._sel.close()
        self._ss.close()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    def _run(self) -> None:
        while self._running:
            for key, _ in self._sel.select(timeout=0.05):
                if key.fileobj is self._ss:
                    try:
                        c, _ = self._ss.accept()
                    except BlockingIOError:
                        continue
                    c.setblocking(True)
                    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    self._conns.append(c)
                    self._sel.register(c, selectors.EVENT_READ)
                else:
                    self._serve(key.fileobj)

    def _serve(self, c: socket.socket) -> None:
        try:
            msg = recv_frame(c)
        except (ConnectionError, OSError, ValueError):
            self._drop(c)
            return
        r = _Reader(msg)
        t = r.i32()
        if t == MSG_CLOSE:
            self._drop(c)
            return
        try:
            res = self.handle(t, r)
        except Exception as e:  # the reference's selector loop ends here (PSAgent.java:188-191)
            self.errors.append(e)
            self._drop(c)
            return
        c.sendall(frame(res))

    def _drop(self, c: socket.socket) -> None:
        try:
            self._sel.unregister(c)
        except (KeyError, ValueError):
            pass
        if c in self._conns:
            self._conns.remove(c)
        c.close()

    def handle(self, t: int, r: _Reader) -> bytes:
        """PSAgent.handle (PSAgent.java:246-285)."""
        if t == MSG_PUSH_REQUEST:
            r.desc()
            data = r.raw(r.i32())
            name = r.raw(r.i32()).decode()
            store, fmt = self.stores[name]
            with self.locks[name]:  # synchronized (store) { store.handlePush(m.getFormat(), data) }
                store.handlePush(fmt, data)
                self.pushes.append((name, data))
            return _i32(MSG_PUSH_RESPONSE) + _i32(1)
        if t == MSG_FETCH_REQUEST:
            name = r.raw(r.i32()).decode()
            store, fmt = self.stores[name]
            rows = read_keys(r, fmt)
            read_keys(r, fmt)  # cols: dense-column rows are fetched whole
            with self.locks[name]:
                out = store.handleFetch(fmt, rows)
            return _i32(MSG_FETCH_RESPONSE) + fmt.write() + _i32(len(out)) + bytes(out) + _name(name)
        raise ValueError(f"message type {t} is not served here")


class PSClient:
    """The worker side of one server connection (blocking request / response)."""

    def __init__(self, address):
        self.sock = socket.create_connection(tuple(address))
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

    def push(self, name: str, fmt: DataDesc, data: bytes) -> bool:
        self.sock.sendall(frame(push_request(name, fmt, data)))
        r = _Reader(recv_frame(self.sock))
        if r.i32() != MSG_PUSH_RESPONSE:
            raise ValueError("unexpected response to a push")
        return r.i32() == 1

    def fetch(self, name: str, fmt: DataDesc, rows: KeyCollection) -> bytes:
        self.sock.sendall(frame(fetch_request(name, fmt, rows)))
        r = _Reader(recv_frame(self.sock))
        if r.i32() != MSG_FETCH_RESPONSE:
            raise ValueError("unexpected response to a fetch")
        r.desc()
        return r.raw(r.i32())

    def close(self) -> None:
        try:
            self.sock.sendall(frame(_i32(MSG_CLOSE)))
        except OSError:
            pass
        finally:
            self.sock.close()
