"""Minimal actor runtime: mailbox + single dispatcher thread + TCP references.

What the reference gets from Akka, rebuilt small:
  * ``Node``: one process-level endpoint (host:port) hosting one actor (the
    master or a worker, like the reference's one actor per JVM).  A TCP server
    thread per inbound connection decodes frames into the actor's mailbox; one
    dispatcher thread delivers them in order, so the actor's ``receive`` is
    single-threaded exactly like an Akka actor's.
  * ``RemoteRef``: ``tell`` encodes and writes to a persistent connection per
    destination -- per sender->receiver FIFO, the ordering the reference's
    tests rely on (SPEC:590, SPEC:721).
  * ``LocalSystem``: the same mailbox semantics with no network, for
    in-process clusters (tests, fault-injection experiments).
"""
from __future__ import annotations

import logging
import queue
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
        self.mailbox: "queue.Queue[Any]" = queue.Queue()
        self._conns: Dict[str, socket.socket] = {}
        self._conn_lock = threading.Lock()
        self._send_locks: Dict[str, threading.Lock] = {}
        self._refs: Dict[str, RemoteRef] = {}
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self.on_send_failure: Optional[Callable[[str, BaseException], None]] = None
        self.on_message: Optional[Callable[[Any], None]] = None  # observer hook (failure detector)
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
        if address == self.address:
            self.mailbox.put(msg)
            return
        if self._stop.is_set():
            return  # a stopped node sends nothing (and opens no new connection)
        frame = wire.encode(msg, self.addr_of)
        with self._conn_lock:
            lock = self._send_locks.setdefault(address, threading.Lock())
        with lock:
            try:
                with self._conn_lock:
                    s = self._conns.get(address)
                if s is None:
                    s = socket.create_connection(parse_addr(address), timeout=10.0)
                    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    s.settimeout(None)
                    with self._conn_lock:
                        if self._stop.is_set():
                            s.close()
                            return
                        self._conns[address] = s
                s.sendall(frame)
            except OSError as e:
                with self._conn_lock:
                    self._conns.pop(address, None)
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
            t = threading.Thread(target=self._read_loop, args=(conn,), name=f"{self.name}-reader", daemon=True)
            t.start()

    def _read_loop(self, conn: socket.socket) -> None:
        try:
            while not self._stop.is_set():
                body = wire.read_frame(conn)
                if body is None:
                    return
                self.mailbox.put(wire.decode(body, self.ref))
        except (OSError, ValueError) as e:
            if not self._stop.is_set():
                log.debug("%s: reader closed: %s", self.name, e)
        finally:
            conn.close()

    def _next_message(self) -> Any:
        poller = self.poller
        while poller is not None and not self._stop.is_set():
            try:
                return self.mailbox.get_nowait()
            except queue.Empty:
                pass
            try:
                st = poller()
            except Exception as e:  # keep the node alive (W:287-299)
                log.exception("%s: error in poller: %s", self.name, e)
                st = None
            if st is None:
                break  # nothing in flight: block on the mailbox
            if not st:
                time.sleep(20e-6)
        return self.mailbox.get()

    def _dispatch_loop(self) -> None:
        while not self._stop.is_set():
            msg = self._next_message()
            if msg is None:
                return
            if self.on_message:
                self.on_message(msg)
            try:
                if hasattr(self.actor, "receive"):
                    self.actor.receive(msg)
                else:
                    self.actor.tell(msg)
            except Exception as e:  # an actor never dies from one message (W:287-299)
                log.exception("%s: error in receive(%s): %s", self.name, type(msg).__name__, e)


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
