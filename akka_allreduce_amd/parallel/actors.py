"""Minimal actor runtime: mailbox + single dispatcher thread + TCP references.

What the reference gets from Akka, rebuilt small:
  * ``Node``: one process-level endpoint (host:port) hosting one actor (the
    master or a worker, like the reference's one actor per JVM).  ONE
    dispatcher thread reads every inbound connection through a selector,
    splits the bytes into frames and runs the actor's ``receive`` on each in
    arrival order -- single-threaded exactly like an Akka actor's, with no
    hand-off between a reader thread and the dispatcher per message (a round
    of the reference's demo is ~7 tiny messages per worker, so the hand-offs
    were most of its time).  Local messages (self-sends, the failure
    detector's notices) go through a mailbox that wakes the selector.
  * ``RemoteRef``: ``tell`` encodes and writes to a persistent connection per
    destination -- per sender->receiver FIFO, the ordering the reference's
    tests rely on (SPEC:590, SPEC:721).
  * ``LocalSystem``: the same mailbox semantics with no network, for
    in-process clusters (tests, fault-injection experiments).
"""
from __future__ import annotations

import collections
import logging
import os
import selectors
import socket
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

from . import wire

log = logging.getLogger("akka_allreduce_amd.actors")


def parse_addr(addr: str) -> Tuple[str, int]:
    host, port = addr.rsplit(":", 1)
    return host, int(port)


class RemoteRef:
    """Reference to the actor hosted by the Node at ``address``."""

    def __init__(self, address: str, node: "Node"):
        self.address = address
        self._node = node

    def tell(self, msg: Any, sender: Any = None) -> None:
        self._node.send(self.address, msg)

    def tell_many(self, msgs: List[Any]) -> None:
        """Several messages in order, written as one batch (one system call)."""
        self._node.send_many(self.address, msgs)

    def tell_frames(self, frames: bytes) -> None:
        """Already-encoded wire frames (the native outbox), in order."""
        self._node.send_frames(self.address, frames)

    def __repr__(self) -> str:
        return f"RemoteRef({self.address})"

    def __eq__(self, other: object) -> bool:
        return isinstance(other, RemoteRef) and other.address == self.address

    def __hash__(self) -> int:
        return hash(self.address)


class Node:
    """TCP endpoint + mailbox + dispatcher for one actor."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, name: str = "node"):
        self.name = name
        self._srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._srv.bind((host, port))
        self._srv.listen(128)
        self.host, self.port = self._srv.getsockname()[:2]
        self.address = f"{host}:{self.port}"
        self.actor: Any = None
        self.aliases: List[Any] = []  # inner objects that stand for this node (e.g. the master logic)
        self._wake_r, self._wake_w = os.pipe()
        os.set_blocking(self._wake_r, False)
        os.set_blocking(self._wake_w, False)
        self._wake_lock = threading.Lock()  # no write into the pipe's fd numbers once they are closed
        self._wake_open = True
        self.mailbox = _Mailbox(self._wake)
        self._accepted: List[socket.socket] = []  # inbound connections the dispatcher has not registered yet
        self._accepted_lock = threading.Lock()
        self._conns: Dict[str, socket.socket] = {}
        self._conn_lock = threading.Lock()
        self._outs: Dict[str, "_Outbound"] = {}  # per destination: socket, pending bytes, flusher state
        self._refs: Dict[str, RemoteRef] = {}
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self.on_send_failure: Optional[Callable[[str, BaseException], None]] = None
        self.on_message: Optional[Callable[[Any], None]] = None  # observer hook (failure detector)
        # Native frame path (a worker on the TCP data plane): connections are
        # read into a native FrameSplitter and ``frame_consumer(splitter,
        # deliver)`` applies its data frames in C++, handing every other frame
        # body to ``deliver`` in order.  Set before start(); not with on_message.
        self.frame_consumer: Optional[Callable[[Any, Callable[[bytes], None]], None]] = None
        # Progress hook run by the dispatcher thread between messages: returns
        # None when there is nothing to drive (the dispatcher then blocks on the
        # mailbox), True after progress, False while work is pending but idle
        # (e.g. the reactive GPU transport's in-flight transfers).
        self.poller: Optional[Callable[[], Optional[bool]]] = None

    # ---- references --------------------------------------------------------------
    def ref(self, address: Optional[str]) -> Any:
        if address is None:
            return None
        if address == self.address:
            return self.aliases[0] if self.aliases else self.actor
        r = self._refs.get(address)
        if r is None:
            r = self._refs[address] = RemoteRef(address, self)
        return r

    def addr_of(self, ref: Any) -> Optional[str]:
        if ref is None:
            return None
        if ref is self.actor or any(ref is a for a in self.aliases):
            return self.address
        if isinstance(ref, RemoteRef):
            return ref.address
        raise TypeError(f"cannot address {ref!r} over the network")

    # ---- lifecycle -----------------------------------------------------------------
    def start(self, actor: Any) -> "Node":
        self.actor = actor
        for target in (self._accept_loop, self._dispatch_loop):
            t = threading.Thread(target=target, name=f"{self.name}-{target.__name__}", daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def _wake(self) -> None:
        with self._wake_lock:
            if not self._wake_open:
                return  # a stopped node
            try:
                os.write(self._wake_w, b"x")
            except BlockingIOError:
                pass  # a full pipe is already a pending wake-up

    def stop(self) -> None:
        self._stop.set()
        self.mailbox.put(None)
        try:
            self._srv.shutdown(socket.SHUT_RDWR)  # wakes the accept loop (close alone does not)
        except OSError:
            pass
        try:
            self._srv.close()
        except OSError:
            pass
        # every access to _conns holds _conn_lock: a sender thread (heartbeats)
        # connecting while the node stops must not change the dict under this
        # loop ("dictionary changed size during iteration" in stop())
        with self._conn_lock:
            conns = list(self._conns.values())
            self._conns.clear()
        for s in conns:
            try:
                s.close()
            except OSError:
                pass

    def join(self, timeout: Optional[float] = None) -> None:
        end = None if timeout is None else time.time() + timeout
        for t in self._threads:
            if t is threading.current_thread():
                continue  # stop() from inside a handler: nothing to wait for here
            t.join(None if end is None else max(0.0, end - time.time()))

    @property
    def stopped(self) -> bool:
        return self._stop.is_set()

    # ---- sending ---------------------------------------------------------------------
    def send(self, address: str, msg: Any) -> None:
        self.send_many(address, [msg])

    def send_many(self, address: str, msgs: List[Any]) -> None:
        """``msgs`` to ``address`` in order: their frames go out in ONE write
        (the receiver's FrameReader splits them), so the per-pair FIFO order
        of the reference holds and a burst costs one system call.

        Never blocks the caller -- which is usually this node's dispatcher,
        the thread that must keep reading the node's sockets.  The write is
        non-blocking (MSG_DONTWAIT); whatever the socket buffer cannot take
        goes to the destination's pending bytes, which a flusher thread writes
        out (later sends queue behind them, so order holds).  Two nodes that
        send each other large payloads from their handlers therefore cannot
        deadlock on full socket buffers."""
        if address == self.address:
            for m in msgs:
                self.mailbox.put(m)
            return
        if self._stop.is_set() or not msgs:
            return  # a stopped node sends nothing (and opens no new connection)
        frame = wire.encode(msgs[0], self.addr_of) if len(msgs) == 1 else \
            b"".join(wire.encode(m, self.addr_of) for m in msgs)
        self.send_frames(address, frame)

    def send_frames(self, address: str, frame: bytes) -> None:
        """Encoded frames to ``address`` (see send_many)."""
        if address == self.address:
            r = wire.FrameReader()
            for body in r.feed(frame):
                self.mailbox.put(wire.decode(body, self.ref))
            return
        if self._stop.is_set() or not frame:
            return
        with self._conn_lock:
            out = self._outs.get(address)
            if out is None:
                out = self._outs[address] = _Outbound()
        with out.lock:
            try:
                if out.sock is None:
                    out.sock = socket.create_connection(parse_addr(address), timeout=10.0)
                    out.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    out.sock.settimeout(None)
                    with self._conn_lock:
                        if self._stop.is_set():
                            out.sock.close()
                            out.sock = None
                            return
                        self._conns[address] = out.sock
                if out.flushing:
                    out.pending += frame  # behind the bytes the flusher still writes
                    return
                try:
                    n = out.sock.send(frame, socket.MSG_DONTWAIT)
                except BlockingIOError:
                    n = 0
                if n == len(frame):
                    return
                out.pending += memoryview(frame)[n:]
                out.flushing = True
            except OSError as e:
                self._send_failed(address, out, e)
                return
        threading.Thread(target=self._flush_pending, args=(address, out), name=f"{self.name}-flush",
                         daemon=True).start()

    def _flush_pending(self, address: str, out: "_Outbound") -> None:
        while True:
            with out.lock:
                if not out.pending or out.sock is None:
                    out.flushing = False
                    out.pending.clear()
                    return
                data, out.pending = out.pending, bytearray()
                sock = out.sock
            try:
                sock.sendall(data)  # blocking, off the dispatcher
            except OSError as e:
                with out.lock:
                    self._send_failed(address, out, e)
                return

    def _send_failed(self, address: str, out: "_Outbound", e: BaseException) -> None:
        """(out.lock held) drop the connection and its pending bytes, report."""
        if out.sock is not None:
            try:
                out.sock.close()
            except OSError:
                pass
        out.sock = None
        out.pending.clear()
        out.flushing = False
        with self._conn_lock:
            self._conns.pop(address, None)
        if self._stop.is_set():
            return  # the node's own shutdown closed the socket under a flusher
        log.warning("%s: send to %s failed: %s", self.name, address, e)
        if self.on_send_failure:
            self.on_send_failure(address, e)

    # ---- receiving -----------------------------------------------------------------
    def _accept_loop(self) -> None:
        while not self._stop.is_set():
            try:
                conn, _ = self._srv.accept()
            except OSError:
                return
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            with self._accepted_lock:
                self._accepted.append(conn)
            self._wake()

    def _deliver(self, msg: Any) -> None:
        if self.on_message:
            self.on_message(msg)
        try:
            if hasattr(self.actor, "receive"):
                self.actor.receive(msg)
            else:
                self.actor.tell(msg)
        except Exception as e:  # an actor never dies from one message (W:287-299)
            log.exception("%s: error in receive(%s): %s", self.name, type(msg).__name__, e)

    def _deliver_body(self, body: bytes) -> None:
        self._deliver(wire.decode(body, self.ref))

    def _new_reader(self) -> Any:
        if self.frame_consumer is not None and self.on_message is None:
            from .._native_loader import load

            return load().FrameSplitter()
        return wire.FrameReader()

    def _poll_timeout(self) -> Optional[float]:
        """Run the progress hook: None -> block until a message, 0 -> progress
        was made (look again at once), else the idle-but-pending back-off."""
        poller = self.poller
        if poller is None:
            return None
        try:
            st = poller()
        except Exception as e:  # keep the node alive (W:287-299)
            log.exception("%s: error in poller: %s", self.name, e)
            st = None
        if st is None:
            return None  # nothing in flight: block
        return 0.0 if st else 20e-6

    def _dispatch_loop(self) -> None:
        sel = selectors.DefaultSelector()
        sel.register(self._wake_r, selectors.EVENT_READ, None)
        inbound: List[socket.socket] = []

        def close(conn: socket.socket) -> None:
            try:
                sel.unregister(conn)
            except (KeyError, ValueError):
                pass
            conn.close()
            if conn in inbound:
                inbound.remove(conn)

        try:
            while not self._stop.is_set():
                while True:  # local messages, in order
                    try:
                        msg = self.mailbox.get_nowait()
                    except IndexError:
                        break
                    if msg is None:
                        return
                    self._deliver(msg)
                timeout = self._poll_timeout()
                if len(self.mailbox):
                    continue  # the poller or a handler posted locally: deliver first
                for key, _ in sel.select(timeout):
                    if key.data is None:  # wake-up: drain, register accepted connections
                        try:
                            while os.read(self._wake_r, 4096):
                                pass
                        except BlockingIOError:
                            pass
                        with self._accepted_lock:
                            new, self._accepted = self._accepted, []
                        for conn in new:
                            sel.register(conn, selectors.EVENT_READ, self._new_reader())
                            inbound.append(conn)
                        continue
                    conn, reader = key.fileobj, key.data
                    try:
                        chunk = conn.recv(1 << 16)
                        if not chunk:
                            close(conn)  # the peer closed the connection
                            continue
                        if isinstance(reader, wire.FrameReader):
                            for body in reader.feed(chunk):
                                self._deliver(wire.decode(body, self.ref))
                        else:  # native splitter: the consumer applies data frames in C++
                            reader.append(chunk)
                            self.frame_consumer(reader, self._deliver_body)
                    except (OSError, ValueError) as e:
                        if not self._stop.is_set():
                            log.debug("%s: reader closed: %s", self.name, e)
                        close(conn)
        finally:
            for conn in list(inbound):
                close(conn)
            sel.close()
            with self._wake_lock:
                self._wake_open = False
                for fd in (self._wake_r, self._wake_w):
                    os.close(fd)


class _Outbound:
    """One destination's connection and the bytes not yet written to it."""

    __slots__ = ("sock", "lock", "pending", "flushing")

    def __init__(self):
        self.sock: Optional[socket.socket] = None
        self.lock = threading.Lock()
        self.pending = bytearray()
        self.flushing = False  # a flusher thread owns the pending bytes


class _Mailbox:
    """A node's local messages (self-sends, notices posted by other threads):
    a thread-safe deque whose ``put`` wakes the dispatcher's selector."""

    def __init__(self, wake: Callable[[], None]):
        self._q: "collections.deque[Any]" = collections.deque()
        self._wake = wake

    def put(self, msg: Any) -> None:
        self._q.append(msg)
        self._wake()

    def get_nowait(self) -> Any:
        return self._q.popleft()  # IndexError when empty

    def __len__(self) -> int:
        return len(self._q)


class LocalRef:
    """In-process reference: tell enqueues into the system's mailbox."""

    def __init__(self, system: "LocalSystem", actor: Any, name: str):
        self.system = system
        self.actor = actor
        self.name = name

    def tell(self, msg: Any, sender: Any = None) -> None:
        self.system.post(self, msg)

    def __repr__(self) -> str:
        return f"LocalRef({self.name})"


class LocalSystem:
    """Deterministic in-process actor system (one global FIFO mailbox).

    ``interceptor(dest_ref, msg) -> bool`` may drop (False) or delay messages
    (by re-posting them later), which is how tests inject stragglers, losses
    and reordering without a network.
    """

    def __init__(self):
        self._q: List[Tuple[LocalRef, Any]] = []
        self.interceptor: Optional[Callable[[LocalRef, Any], bool]] = None
        self.delivered = 0

    def spawn(self, actor: Any, name: str) -> LocalRef:
        return LocalRef(self, actor, name)

    def post(self, ref: LocalRef, msg: Any) -> None:
        self._q.append((ref, msg))

    def run(self, max_messages: int = 10_000_000) -> int:
        n = 0
        while self._q and n < max_messages:
            ref, msg = self._q.pop(0)
            if self.interceptor is not None and not self.interceptor(ref, msg):
                continue
            ref.actor.receive(msg)
            n += 1
        self.delivered += n
        return n
