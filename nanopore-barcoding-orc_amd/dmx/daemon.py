"""Resident `cutadapt` server for the unchanged 02_cutadapt_loop.sh.

The script calls `cutadapt` 13 times (`scripts/02_cutadapt_loop.sh:64-72,91-103`); per call a
fresh process pays interpreter + numpy start (~0.14 s), HIP runtime and context start
(0.1-0.2 s) and HIP teardown at exit (~0.1 s), more than the 12 round-2 calls' own work. The
drop-in `bin/cutadapt` is therefore a thin client: it forwards argv, cwd and the DMX_*
environment over a UNIX socket to this server, which keeps the library, the HIP runtime and one
context per device loaded and runs `dmx.cli.run` in-process, then returns the call's stdout,
stderr and exit status. The first call starts the server; it exits after `idle` seconds
without a request. `DMX_DAEMON=0` makes every call run in its own process (the behaviour is
the same either way; tests cover both).

Isolation: one server per (user, checkout, SLURM job, GPU visibility, library build). The socket
name hashes SLURM_JOB_ID, the GPU-visibility variables (HIP/ROCR/CUDA_VISIBLE_DEVICES,
GPU_DEVICE_ORDINAL) and the library selectors (DMX_LIBDMX, DMX_LIBDIR, DMX_DEBUG_BOUNDS), so a job never talks to another job's server (which would use the other
job's GPUs and die with it, `04_cleaning_primers.sh:4,7` is a 96-task array), and the server,
spawned by its first client, sees exactly the devices its callers see. A request is served
with only its own DMX_* variables; contexts are cached per (devices, dmx_open-time switches).
One request runs at a time: a call that arrives while another is running is answered "busy"
and the client runs it in its own process instead of queueing. After a GPU error the server
closes its contexts and exits, so the next call starts a fresh process.

Protocol: request = u32 length + JSON {"argv", "cwd", "env"}; reply = frames u8 tag + u32 length
+ payload, tags b"o" (stdout bytes), b"e" (stderr bytes), b"x" (exit status as text), or a
single b"b" frame (busy: run in-process)."""
from __future__ import annotations

import json
import os
import socket
import struct
import sys
import tempfile
import threading
import time
import zlib

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# variables that decide which GPUs a process sees (and so which server may serve it)
VISIBILITY_ENV = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
                  "GPU_DEVICE_ORDINAL")
# variables that decide which libdmx / libdmx_io build a process loads (read once at import by
# dmx/lib.py and dmx/nio.py, so a server cannot switch them per request), and the memory budget
# libdmx_io's buffers are sized to at load (nio.memory_budget_bytes): a call that sets them (A/B
# or sanitizer builds, a budget) gets a server of its own
LIBRARY_ENV = ("DMX_LIBDMX", "DMX_LIBDIR", "DMX_DEBUG_BOUNDS", "DMX_MEM_BUDGET_MB")


def socket_path(env=None) -> str:
    """One server per user, checkout, SLURM job and GPU visibility; the same rule as the
    client's (bin/cutadapt _sock_path)."""
    env = os.environ if env is None else env
    if env.get("DMX_DAEMON_SOCK"):
        return env["DMX_DAEMON_SOCK"]
    tmp = "/tmp"
    for k in ("TMPDIR", "TEMP", "TMP"):
        d = env.get(k)
        if d and os.path.isdir(d):
            tmp = d
            break
    scope = "|".join([PKG, env.get("SLURM_JOB_ID", "")] +
                     [f"{k}={env.get(k, '<unset>')}" for k in VISIBILITY_ENV + LIBRARY_ENV])
    return os.path.join(tmp, f"dmx-{os.getuid()}-{zlib.crc32(scope.encode()):08x}.sock")


def _recv_exact(conn, n: int) -> bytes:
    buf = b""
    while len(buf) < n:
        chunk = conn.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("peer closed")
        buf += chunk
    return buf


def _frame(tag: bytes, payload: bytes) -> bytes:
    return tag + struct.pack("<I", len(payload)) + payload


class _Captured:
    """fd-level capture of stdout/stderr (Python and native writers) for one request."""

    def __enter__(self):
        sys.stdout.flush()
        sys.stderr.flush()
        self.files = [tempfile.TemporaryFile(), tempfile.TemporaryFile()]
        self.saved = [os.dup(1), os.dup(2)]
        os.dup2(self.files[0].fileno(), 1)
        os.dup2(self.files[1].fileno(), 2)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        sys.stderr.flush()
        os.dup2(self.saved[0], 1)
        os.dup2(self.saved[1], 2)
        for fd in self.saved:
            os.close(fd)
        self.out = []
        for f in self.files:
            f.seek(0)
            self.out.append(f.read())
            f.close()
        return False


def _handle(conn) -> bool:
    """Serve one request; returns True when the server must exit (a GPU error: its contexts
    may hold a sticky HIP error)."""
    from . import cli, lib   # imported once, in the server process
    n = struct.unpack("<I", _recv_exact(conn, 4))[0]
    req = json.loads(_recv_exact(conn, n).decode())
    # the caller's directory and exactly its DMX_* settings for this call
    for k in [k for k in os.environ if k.startswith("DMX_")]:
        del os.environ[k]
    os.environ.update({k: v for k, v in req.get("env", {}).items() if k.startswith("DMX_")})
    code = 1
    fatal = False
    with _Captured() as cap:
        try:
            os.chdir(req["cwd"])
            code = cli.run(req["argv"], keep_contexts=True)
        except SystemExit as e:            # argparse, unsupported options
            code = e.code if isinstance(e.code, int) else (0 if e.code is None else 1)
            if isinstance(e.code, str):
                print(e.code, file=sys.stderr)
        except lib.DmxError as e:
            print(f"cutadapt (dmx): GPU error: {e}", file=sys.stderr)
            code = 1
            fatal = True
        except Exception as e:             # keep serving; the caller sees the failure
            print(f"cutadapt (dmx): error: {type(e).__name__}: {e}", file=sys.stderr)
            code = 1
    conn.sendall(_frame(b"o", cap.out[0]) + _frame(b"e", cap.out[1]) +
                 _frame(b"x", str(int(code)).encode()))
    return fatal


def _admit(busy, state) -> bool:
    """Take the one-call lock for an accepted connection.  One call runs at a time; others are
    answered "busy" and run in-process.  So is a call accepted after a worker hit a GPU error
    (state["fatal"], set just before that worker released the lock): it must not run on contexts
    that may hold a sticky HIP error, and the accept loop exits right after."""
    if not busy.acquire(blocking=False):
        return False
    if state["fatal"]:
        busy.release()
        return False
    return True


def serve(path: str, idle: float):
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    try:
        srv.bind(path)
    except OSError:
        return                                # another server owns the path
    ino = os.stat(path).st_ino
    os.chmod(path, 0o600)
    srv.listen(16)
    srv.settimeout(0.25)
    home = os.getcwd()
    busy = threading.Lock()
    state = {"last": time.monotonic(), "fatal": False}

    def work(conn):
        try:
            with conn:
                try:
                    state["fatal"] |= _handle(conn)
                except (ConnectionError, OSError, ValueError):
                    pass
            os.chdir(home)
        finally:
            state["last"] = time.monotonic()
            busy.release()

    worker = None
    try:
        while not state["fatal"]:
            try:
                conn, _ = srv.accept()
            except socket.timeout:
                if not busy.locked() and time.monotonic() - state["last"] > idle:
                    break
                continue
            if not _admit(busy, state):
                with conn:
                    try:   # take the request off the wire first, so the client sees the reply
                        conn.settimeout(2.0)
                        _recv_exact(conn, struct.unpack("<I", _recv_exact(conn, 4))[0])
                        conn.sendall(_frame(b"b", b""))
                    except (OSError, ConnectionError, struct.error):
                        pass
                continue
            worker = threading.Thread(target=work, args=(conn,), daemon=True)
            worker.start()
        if worker is not None:
            worker.join()
    finally:
        srv.close()
        try:   # only our own socket: a later server may have bound the path since
            if os.stat(path).st_ino == ino:
                os.unlink(path)
        except OSError:
            pass
        from . import cli
        cli.close_cached_contexts()


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else socket_path()
    idle = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    serve(path, idle)


if __name__ == "__main__":
    main()
