"""Resident `cutadapt` server isolation (dmx/daemon.py, bin/cutadapt; CPU only).

The reference runs the demux from a 96-task SLURM array (scripts/04_cleaning_primers.sh:4,7) and
calls `cutadapt` 13 times per sample (scripts/02_cutadapt_loop.sh:64-72,91-103).  A resident
server must therefore never serve a call from another job or with another GPU visibility, must
apply exactly the calling process's DMX_* settings, must not queue a call behind another one,
and must exit after a GPU error.  The CLI itself is replaced by a stub here (no GPU)."""
import importlib.machinery
import importlib.util
import json
import os
import socket
import struct
import threading
import time

import pytest

from dmx import cli, daemon, lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLIENT = os.path.join(ROOT, "nanopore-barcoding-orc_amd", "bin", "cutadapt")


def _client_module():
    loader = importlib.machinery.SourceFileLoader("dmx_cutadapt_client", CLIENT)
    spec = importlib.util.spec_from_loader("dmx_cutadapt_client", loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod


def _scoped(monkeypatch, **env):
    monkeypatch.delenv("DMX_DAEMON_SOCK", raising=False)
    for k in daemon.VISIBILITY_ENV + daemon.LIBRARY_ENV + ("SLURM_JOB_ID",):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)


def test_socket_scope_by_gpu_visibility_and_job(monkeypatch):
    client = _client_module()
    paths = {}
    for name, env in {"plain": {}, "hip0": {"HIP_VISIBLE_DEVICES": "0"},
                      "hip1": {"HIP_VISIBLE_DEVICES": "1"},
                      "rocr1": {"ROCR_VISIBLE_DEVICES": "1"},
                      "job7": {"SLURM_JOB_ID": "7"},
                      "job8": {"SLURM_JOB_ID": "8"},
                      "job7_hip1": {"SLURM_JOB_ID": "7", "HIP_VISIBLE_DEVICES": "1"},
                      # another libdmx / libdmx_io build (A/B, sanitizers): its own server
                      "libdmx_ab": {"DMX_LIBDMX": "/x/libdmx_ab.so"},
                      "libdir_asan": {"DMX_LIBDIR": "/x/build/asan"}}.items():
        _scoped(monkeypatch, **env)
        paths[name] = client._sock_path()
        assert paths[name] == daemon.socket_path(), "client and server disagree on the socket"
    assert len(set(paths.values())) == len(paths)
    # an explicit socket still wins (tests, DMX_DAEMON_SOCK)
    monkeypatch.setenv("DMX_DAEMON_SOCK", "/tmp/x.sock")
    assert client._sock_path() == daemon.socket_path() == "/tmp/x.sock"


def _request(path, argv, env):
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.connect(path)
    req = json.dumps({"argv": argv, "cwd": os.getcwd(), "env": env}).encode()
    s.sendall(struct.pack("<I", len(req)) + req)
    frames = {}
    with s:
        while True:
            tag = s.recv(1)
            if not tag:
                break
            n = struct.unpack("<I", s.recv(4))[0]
            payload = b""
            while len(payload) < n:
                payload += s.recv(n - len(payload))
            frames[tag] = payload
            if tag in (b"x", b"b"):
                break
    return frames


def _wait_socket(path, t=10.0):
    end = time.monotonic() + t
    while not os.path.exists(path):
        assert time.monotonic() < end, "server did not start"
        time.sleep(0.01)


@pytest.fixture
def server(tmp_path, monkeypatch):
    """serve() in a thread of this process with cli.run replaced by a stub."""
    calls = []
    gate = {"ev": None}

    def fake_run(argv, keep_contexts=False):
        calls.append((list(argv), {k: v for k, v in os.environ.items() if k.startswith("DMX_")}))
        if argv and argv[0] == "block":
            gate["ev"].wait(10)
        if argv and argv[0] == "gpu-error":
            raise lib.DmxError("sticky HIP error")
        os.write(1, b"stdout of " + (argv[0] if argv else "").encode() + b"\n")
        return 0

    monkeypatch.setattr(cli, "run", fake_run)
    path = str(tmp_path / "d.sock")
    th = threading.Thread(target=daemon.serve, args=(path, 3.0), daemon=True)
    th.start()
    _wait_socket(path)
    yield path, calls, gate, th
    if gate["ev"] is not None:
        gate["ev"].set()
    th.join(10)


def test_request_env_is_exactly_the_callers(server, monkeypatch):
    path, calls, _, _ = server
    monkeypatch.setenv("DMX_SERVER_START_ONLY", "1")   # present in the server's own environment
    f1 = _request(path, ["a"], {"DMX_BATCH_MB": "64", "DMX_GPUS": "2", "OTHER": "x"})
    f2 = _request(path, ["b"], {"DMX_NO_SCREEN": "1"})
    assert f1[b"x"] == b"0" and f2[b"x"] == b"0"
    assert b"stdout of a" in f1[b"o"]
    assert calls[0][1] == {"DMX_BATCH_MB": "64", "DMX_GPUS": "2"}
    assert calls[1][1] == {"DMX_NO_SCREEN": "1"}     # nothing left over from the first call


def test_concurrent_call_is_answered_busy(server):
    path, calls, gate, _ = server
    gate["ev"] = threading.Event()
    res = {}
    t = threading.Thread(target=lambda: res.setdefault("first", _request(path, ["block"], {})))
    t.start()
    end = time.monotonic() + 10
    while not calls:
        assert time.monotonic() < end
        time.sleep(0.01)
    second = _request(path, ["second"], {})
    assert b"b" in second and b"x" not in second     # the client runs it in-process instead
    gate["ev"].set()
    t.join(10)
    assert res["first"][b"x"] == b"0"
    assert [c[0][0] for c in calls] == ["block"]


def test_gpu_error_ends_the_server(server):
    path, calls, _, th = server
    f = _request(path, ["gpu-error"], {})
    assert f[b"x"] == b"1"
    th.join(10)
    assert not th.is_alive()
    assert not os.path.exists(path)


def test_call_after_a_gpu_error_is_not_admitted():
    """a connection accepted between a worker's GPU error and the accept loop's exit
    gets the lock but must be answered "busy" (run in-process), not served."""
    busy = threading.Lock()
    state = {"fatal": False}
    assert daemon._admit(busy, state)
    assert not daemon._admit(busy, state)     # a call is running
    busy.release()
    state["fatal"] = True                     # the worker's GPU error, lock released after it
    assert not daemon._admit(busy, state)
    assert not busy.locked()                  # the lock is not leaked


def test_server_unlinks_only_its_own_socket(tmp_path, monkeypatch):
    """A server whose path was taken over by a newer server leaves the newer socket alone."""
    monkeypatch.setattr(cli, "run", lambda argv, keep_contexts=False: 0)
    path = str(tmp_path / "d.sock")
    th = threading.Thread(target=daemon.serve, args=(path, 0.5), daemon=True)
    th.start()
    _wait_socket(path)
    os.unlink(path)
    other = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    other.bind(path)
    th.join(10)
    assert os.path.exists(path)
    other.close()


def test_cached_contexts_keyed_by_open_time_switches(monkeypatch):
    opened = []

    class FakeCtx:
        def __init__(self, devs):
            self.devs = devs
            self.closed = False

        def close(self):
            self.closed = True

    monkeypatch.setattr(lib, "open_group", lambda devs: opened.append(FakeCtx(devs)) or
                        [opened[-1]])
    cli.close_cached_contexts()

    def ctx_for(env):
        for k in cli.OPEN_TIME_ENV:
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        return cli.cached_group([0])[0]

    a = ctx_for({})
    assert ctx_for({}) is a
    b = ctx_for({"DMX_NO_SCREEN": "1"})
    assert b is not a and a.closed
    cli.close_cached_contexts()
