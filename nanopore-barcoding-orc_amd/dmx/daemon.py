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

Protocol: request = u32 length + JSON {"argv", "cwd", "env"}; reply = frames u8 tag + u32 length
+ payload, tags b"o" (stdout bytes), b"e" (stderr bytes), b"x" (exit status as text)."""
from __future__ import annotations

import json
import os
import socket
import struct
import sys
import tempfile
import zlib

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def socket_path() -> str:
    """One server per user and checkout (a different tree never answers for this one); the
    same rule as the client's (bin/cutadapt _sock_path)."""
    env = os.environ.get("DMX_DAEMON_SOCK")
    if env:
        return env
    tmp = "/tmp"
    for k in ("TMPDIR", "TEMP", "TMP"):
        d = os.environ.get(k)
        if d and os.path.isdir(d):
            tmp = d
            break
    return os.path.join(tmp, f"dmx-{os.getuid()}-{zlib.crc32(PKG.encode()):08x}.sock")


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


def _handle(conn, base_env: dict):
    from . import cli, lib   # imported once, in the server process
    n = struct.unpack("<I", _recv_exact(conn, 4))[0]
    req = json.loads(_recv_exact(conn, n).decode())
    # the caller's directory and DMX_* settings for this call only
    for k in [k for k in os.environ if k.startswith("DMX_") and k not in base_env]:
        del os.environ[k]
    os.environ.update({k: v for k, v in base_env.items() if k.startswith("DMX_")})
    os.environ.update({k: v for k, v in req.get("env", {}).items() if k.startswith("DMX_")})
    code = 1
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
        except Exception as e:             # keep serving; the caller sees the failure
            print(f"cutadapt (dmx): error: {type(e).__name__}: {e}", file=sys.stderr)
            code = 1
    conn.sendall(_frame(b"o", cap.out[0]) + _frame(b"e", cap.out[1]) +
                 _frame(b"x", str(int(code)).encode()))


def serve(path: str, idle: float):
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    try:
        srv.bind(path)
    except OSError:
        return                                # another server owns the path
    os.chmod(path, 0o600)
    srv.listen(8)
    srv.settimeout(idle)
    base_env = dict(os.environ)
    home = os.getcwd()
    try:
        while True:
            try:
                conn, _ = srv.accept()
            except socket.timeout:
                break
            with conn:
                try:
                    _handle(conn, base_env)
                except (ConnectionError, OSError, ValueError):
                    pass
            os.chdir(home)
    finally:
        srv.close()
        try:
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
