"""Host collectives for one process per GPU, without a framework.

bench.py's multi-GPU path and the two-process tests use this instead of torch.distributed:
importing the PyTorch wheel maps the HIP runtime, HSA runtime and RCCL it bundles (ROCm 7.0),
and libgprx -- linked against /opt/rocm (7.2) by soname -- would then either bind torch's copies
(torch imported first) or sit beside a second, idle copy of every runtime (libgprx first).  With
these sockets the process maps exactly one runtime, /opt/rocm's, at every world size
(gpr_amd.runtime_info() records which).

The collectives are the few the library and the bench need around the device work:
* `allgather(bytes)`: the all-gather `gprx_ctx_create_peer` bootstraps with (IPC handles, status
  agreement, host barriers) -- `allgather_fn()` adapts it to the C callback;
* `barrier()`, `max(x)`, `min(x)`, `broadcast(bytes)` for the bench's timing contract.
Star topology through rank 0 over TCP on the loopback (one node, as the bench contract says);
the data path of the sharded fit never goes through it (device-initiated IPC stores over xGMI,
DESIGN.md section 6).

Rendezvous: under torch.distributed.run (or bench.py's own spawner) every rank has the
launcher as its parent and the same MASTER_PORT (which a torch launcher's own store occupies).
Rank 0 listens on an ephemeral port of the loopback and publishes "<port> <token>" in
/tmp/gprx_coll_<parent pid>_<MASTER_PORT>_<restart>.port (mode 0600); the other ranks wait for
that file.  GPRX_COLL_PORT fixes the port instead (rank 0 binds it, the others connect to it; the
token is then GPRX_COLL_TOKEN, empty by default).  The group binds 127.0.0.1 (one node, the
bench contract) unless GPRX_COLL_ADDR names another address.

Admission: a connecting rank announces its rank and the launch's token; rank 0 drops (closes and
keeps waiting past) a connection with a wrong token, a rank outside 1..world-1, a rank that has
already joined, or no announcement within 10 s -- a stray connection cannot take a rank's slot or
hang the group.  This socket carries the IPC handles the peer context bootstraps with.
"""
import os
import socket
import struct
import tempfile
import time

_HDR = struct.Struct("<q")


def _send(sock, data):
    sock.sendall(_HDR.pack(len(data)) + data)


def _recv_exact(sock, n):
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("gpr_amd.hostcoll: peer closed the connection")
        got += k
    return bytes(buf)


def _recv(sock):
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    return _recv_exact(sock, n)


class SocketGroup:
    """`world` processes on one host; rank 0 is the hub."""

    def __init__(self, rank, world, addr="127.0.0.1", port=None, port_file=None, timeout=300.0, op_timeout=None,
                 token=None):
        if world < 1 or not (0 <= rank < world):
            raise ValueError("SocketGroup: need 0 <= rank < world")
        self.rank, self.world = rank, world
        # a collective a peer never joins raises instead of blocking for ever (GPRX_COLL_TIMEOUT_S)
        if op_timeout is None:
            op_timeout = float(os.environ.get("GPRX_COLL_TIMEOUT_S", "900"))
        self._conns = {}
        self._sock = None
        self._port_file = None
        if world == 1:
            return
        deadline = time.monotonic() + timeout
        if token is None:  # (a fixed port: the caller's token; a port file: one per launch, below)
            token = os.environ.get("GPRX_COLL_TOKEN", "") if (port is not None or not port_file) else None
        if rank == 0:
            if token is None:
                token = os.urandom(16).hex()
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, int(port) if port else 0))
            srv.listen(world)
            if port_file:
                fd, tmp = tempfile.mkstemp(dir=os.path.dirname(port_file) or ".")
                with os.fdopen(fd, "w") as f:  # (mkstemp: mode 0600)
                    f.write(f"{srv.getsockname()[1]} {token}")
                os.replace(tmp, port_file)
                self._port_file = port_file
            try:
                while len(self._conns) < world - 1:
                    srv.settimeout(max(0.1, deadline - time.monotonic()))
                    try:
                        c, _ = srv.accept()
                    except socket.timeout:
                        raise TimeoutError(f"gpr_amd.hostcoll: {len(self._conns) + 1} of {world} ranks arrived "
                                           f"within {timeout:.0f} s")
                    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    r = self._admit(c, token)
                    if r is None:
                        c.close()
                        continue
                    c.settimeout(op_timeout)
                    self._conns[r] = c
            finally:
                srv.close()
                if self._port_file:  # every rank has connected (or the group failed): done with it
                    try:
                        os.remove(self._port_file)
                    except OSError:
                        pass
                    self._port_file = None
        else:
            while True:
                try:
                    if port is None:
                        with open(port_file) as f:
                            txt = f.read().split()
                        if len(txt) != 2:
                            raise FileNotFoundError(port_file)
                        p, token = int(txt[0]), txt[1]
                    else:
                        p = int(port)
                    s = socket.create_connection((addr, p), timeout=5.0)
                    break
                except (OSError, ValueError):
                    if time.monotonic() > deadline:
                        raise TimeoutError(f"gpr_amd.hostcoll: rank {rank} could not reach rank 0 within "
                                           f"{timeout:.0f} s")
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.settimeout(op_timeout)
            tok = (token or "").encode()
            s.sendall(struct.pack("<ii", rank, len(tok)) + tok)
            self._sock = s

    def _admit(self, c, token):
        """The announced rank of a new connection, or None to drop it (see the module notes)."""
        try:
            c.settimeout(10.0)
            r, nt = struct.unpack("<ii", _recv_exact(c, 8))
            if not (0 <= nt <= 256):
                return None
            tok = _recv_exact(c, nt).decode(errors="replace") if nt else ""
        except (OSError, ConnectionError, struct.error):
            return None
        if tok != (token or "") or not (1 <= r < self.world) or r in self._conns:
            return None
        return r

    @classmethod
    def from_env(cls, timeout=300.0):
        """The group of a torch.distributed.run launch (RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT)
        or of any launcher that sets them; GPRX_COLL_PORT overrides the rendezvous file."""
        rank = int(os.environ.get("RANK", "0"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        addr = os.environ.get("GPRX_COLL_ADDR", "127.0.0.1")
        port = os.environ.get("GPRX_COLL_PORT")
        port_file = None
        if port is None:
            tag = "{}_{}_{}".format(os.getppid(), os.environ.get("MASTER_PORT", "0"),
                                    os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
            port_file = os.path.join(tempfile.gettempdir(), f"gprx_coll_{tag}.port")
            if rank == 0 and os.path.exists(port_file):
                os.remove(port_file)  # (a stale file of an earlier launch by the same parent)
        return cls(rank, world, addr=addr, port=port, port_file=port_file, timeout=timeout)

    # ---- collectives ---------------------------------------------------------------------
    def allgather(self, data):
        """Every rank's bytes, in rank order (lengths may differ)."""
        data = bytes(data)
        if self.world == 1:
            return [data]
        if self.rank == 0:
            parts = [data] + [_recv(self._conns[r]) for r in range(1, self.world)]
            blob = b"".join(_HDR.pack(len(p)) + p for p in parts)
            for r in range(1, self.world):
                self._conns[r].sendall(blob)
            return parts
        _send(self._sock, data)
        return [_recv(self._sock) for _ in range(self.world)]

    def barrier(self):
        self.allgather(b"")

    def broadcast(self, data=None):
        """Rank 0's bytes on every rank."""
        return self.allgather(bytes(data or b"") if self.rank == 0 else b"")[0]

    def max(self, x):
        return max(struct.unpack("<d", p)[0] for p in self.allgather(struct.pack("<d", float(x))))

    def min(self, x):
        return min(struct.unpack("<d", p)[0] for p in self.allgather(struct.pack("<d", float(x))))

    def allgather_fn(self):
        """This group as a gprx_allgather_fn (include/gprx.h: every rank passes the same byte
        count) for gpr_amd.Context(peer=(rank, world, fn))."""
        import ctypes

        def fn(user, send, nbytes, recv):
            try:
                parts = self.allgather(ctypes.string_at(send, nbytes) if nbytes else b"")
                if any(len(p) != nbytes for p in parts):
                    return 1
                if nbytes:
                    ctypes.memmove(recv, b"".join(parts), nbytes * self.world)
                return 0
            except Exception:  # reported to the library as a failed collective
                return 1
        return fn

    def close(self):
        for c in self._conns.values():
            try:
                c.close()
            except OSError:
                pass
        self._conns = {}
        if self._sock is not None:
            try:
                self._sock.close()
            except OSError:
                pass
            self._sock = None
        if self._port_file:
            try:
                os.remove(self._port_file)
            except OSError:
                pass
            self._port_file = None
