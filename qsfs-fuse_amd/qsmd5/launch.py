"""Rank processes for bench.py / bench_config5.py without an external launcher.

The driver runs ``python bench.py --gpus N`` bare; torch.distributed.run is
not in front of it.  spawn_ranks() makes the same
one-process-per-GPU layout torchrun would: N fresh child processes running the
same script with RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE /
MASTER_ADDR / MASTER_PORT set, so every rank initialises its own GPU and RCCL
communicator.  The parent makes no torch.cuda or HIP call at all (this module
imports neither torch nor libqsmd5), and it never replaces itself with a child
(no exec): it waits for the children and exits with their worst status.

Output: rank 0's stdout is the parent's stdout (the one JSON line); the other
ranks' stdout goes to the parent's stderr with their logs, so stdout carries
rank 0's line only.  If a rank fails, the others get ``grace_s`` seconds to
finish (a collective they are blocked in usually fails by itself), then
SIGTERM, then SIGKILL -- each by its exact PID.  A SIGTERM / SIGINT to the
parent is passed on to every child the same way.
"""
import os
import signal
import socket
import subprocess
import sys
import time

__all__ = ["free_port", "launched", "spawn_ranks", "worst_status"]


def free_port():
    """A TCP port on 127.0.0.1 that was free a moment ago (the rendezvous)."""
    s = socket.socket()
    try:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
    finally:
        s.close()


def launched():
    """True when a launcher (torchrun, or spawn_ranks) already set the rank env."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def worst_status(codes):
    """One exit status for the job: 0 if every rank exited 0, else the first
    failing rank's status in rank order (a rank killed by signal s counts as
    128 + s, as a shell reports it)."""
    for c in codes:
        if c is None:
            return 1
        if c != 0:
            return 128 - c if c < 0 else c
    return 0


def _stop(procs, sig):
    for p in procs:
        if p.poll() is None:
            try:
                p.send_signal(sig)
            except OSError:
                pass


def spawn_ranks(script, argv, nproc, env_extra=None, grace_s=60.0, python=None):
    """Run ``python script *argv`` as nproc ranks on this node; returns the
    job's exit status: the status of the first rank seen failing (the ranks
    stopped after it do not mask it), else 0."""
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    port = free_port()
    base = dict(os.environ)
    base.update(env_extra or {})
    base.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                 "WORLD_SIZE": str(nproc), "LOCAL_WORLD_SIZE": str(nproc),
                 "GROUP_RANK": "0", "NODE_RANK": "0", "QSMD5_SPAWNED_BY": "bench"})
    procs = []
    prev = {}

    def forward(signum, _frame):
        _stop(procs, signum)

    for s in (signal.SIGTERM, signal.SIGINT):
        try:
            prev[s] = signal.signal(s, forward)
        except ValueError:  # not the main thread: no handler, the children still end with us
            pass
    try:
        for r in range(nproc):
            env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen(
                [python or sys.executable, "-u", script] + list(argv), env=env,
                stdout=None if r == 0 else sys.stderr.fileno()))
        failed_at, first_bad = None, None
        while True:
            codes = [p.poll() for p in procs]
            if failed_at is None and any(c not in (None, 0) for c in codes):
                failed_at = time.monotonic()
                bad = [r for r, c in enumerate(codes) if c not in (None, 0)]
                first_bad = codes[bad[0]]  # the root cause, not the ranks stopped after it
                print("spawn_ranks: rank %s exited with %s; the other ranks get %.0f s"
                      % (bad, [codes[r] for r in bad], grace_s), file=sys.stderr, flush=True)
            if all(c is not None for c in codes):
                break
            if failed_at is not None and time.monotonic() - failed_at > grace_s:
                _stop(procs, signal.SIGTERM)
                t_kill = time.monotonic() + 10.0
                while time.monotonic() < t_kill and any(p.poll() is None for p in procs):
                    time.sleep(0.1)
                _stop(procs, signal.SIGKILL)
                for p in procs:
                    p.wait()
                break
            time.sleep(0.05)
        if first_bad is not None:
            return worst_status([first_bad])
        return worst_status([p.returncode for p in procs])
    finally:
        _stop(procs, signal.SIGKILL)  # only children still running (an exception above)
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                pass
        for s, h in prev.items():
            signal.signal(s, h)
