"""One process per GPU without torch: a launcher and a file rendezvous.

``spawn(n, argv)`` starts ``n`` fresh child processes of this interpreter
(``python <argv>``) BEFORE the parent touches the GPU, each with
``RANK``/``LOCAL_RANK``/``WORLD_SIZE`` and a private rendezvous directory in
``ZF_RDZV_DIR``; it returns the worst child exit status.  The same program
also runs under ``python -m torch.distributed.run --nproc-per-node N`` (the
driver's launcher): then the ranks already have the env, and
``FileRendezvous.from_env`` derives a directory shared by the ranks of that
launch from ``MASTER_PORT`` and the launching agent's pid.

The rendezvous is the control plane only — the RCCL unique id broadcast,
barriers outside timed regions, and the max over ranks of a few floats —
through atomically renamed files in a node-local directory.  Data-path
collectives go through RCCL (``dist.RcclCommunicator``)."""

from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path
from typing import Any, List, Optional, Sequence


def spawn(n: int, argv: Sequence[str], env: Optional[dict] = None, timeout: Optional[float] = None,
          grace: float = 20.0) -> int:
    """Run ``python argv`` as ranks 0..n-1 (one process per GPU) and wait.

    Returns 0 if every rank exited 0, else the first non-zero status (a
    negative signal number is mapped to 128 + signal, as a shell would).
    When one rank fails, the others get ``grace`` seconds to end on their
    own (and report their own error) before they are terminated: a rank
    blocked in the rendezvous on the failed one would otherwise wait out
    its timeout.  The parent never initialises the GPU, so exec-free
    process creation is safe on this pool."""
    if n < 1:
        raise ValueError("n must be >= 1")
    rdzv = tempfile.mkdtemp(prefix="zf_rdzv_")
    procs: List[subprocess.Popen] = []
    try:
        for r in range(n):
            e = dict(os.environ if env is None else env)
            e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                     ZF_RDZV_DIR=rdzv)
            procs.append(subprocess.Popen([sys.executable, *argv], env=e))
        deadline = None if timeout is None else time.monotonic() + timeout
        rc = 0
        for p in procs:
            left = None if deadline is None else max(0.0, deadline - time.monotonic())
            try:
                s = p.wait(timeout=left)
            except subprocess.TimeoutExpired:
                s = 124
            if s != 0 and rc == 0:
                rc = s if s > 0 else 128 - s
            if s != 0:  # one rank failed: the others would wait for it forever
                until = time.monotonic() + grace
                for q in procs:
                    try:
                        q.wait(timeout=max(0.0, until - time.monotonic()))
                    except subprocess.TimeoutExpired:
                        q.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        return rc
    finally:
        shutil.rmtree(rdzv, ignore_errors=True)


class RendezvousTimeout(RuntimeError):
    pass


class FileRendezvous:
    """Control-plane exchange among the ``world`` ranks of one node."""

    def __init__(self, path, rank: int, world: int, timeout: float = 600.0, poll: float = 2e-4):
        self.path = Path(path)
        self.path.mkdir(parents=True, exist_ok=True)
        self.rank, self.world = int(rank), int(world)
        self.timeout = timeout
        self.poll = poll
        self._seq = 0

    @classmethod
    def from_env(cls, **kw) -> "FileRendezvous":
        """Rank/world from the env; the directory from ``ZF_RDZV_DIR`` (set by
        ``spawn``) or, under torch.distributed.run, from MASTER_PORT and the
        parent pid shared by the ranks of one launch."""
        rank = int(os.environ.get("RANK", "0"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        d = os.environ.get("ZF_RDZV_DIR")
        if not d:
            port = os.environ.get("MASTER_PORT", "0")
            run = os.environ.get("TORCHELASTIC_RUN_ID", "none")
            ppid = os.getppid()
            d = os.path.join(tempfile.gettempdir(), f"zf_rdzv_{port}_{run}_{ppid}_{_start_time(ppid)}")
        return cls(d, rank, world, **kw)

    # -- primitives ----------------------------------------------------------------
    def _write(self, name: str, payload: bytes) -> None:
        tmp = self.path / f".{name}.{self.rank}.tmp"
        tmp.write_bytes(payload)
        os.replace(tmp, self.path / name)

    def _wait(self, name: str) -> bytes:
        f = self.path / name
        t0 = time.monotonic()
        delay = self.poll
        while not f.exists():
            if time.monotonic() - t0 > self.timeout:
                raise RendezvousTimeout(f"rank {self.rank}: no {name} after {self.timeout:.0f} s")
            time.sleep(delay)
            delay = min(delay * 2, 0.01)
        return f.read_bytes()

    def _tag(self, tag: Optional[str]) -> str:
        self._seq += 1
        return f"{self._seq:06d}_{tag or 'x'}"

    def allgather(self, value: Any, tag: Optional[str] = None) -> List[Any]:
        """Every rank's JSON-serialisable ``value``, in rank order."""
        t = self._tag(tag)
        self._write(f"{t}.{self.rank}", json.dumps(value).encode())
        return [json.loads(self._wait(f"{t}.{r}")) for r in range(self.world)]

    def allgather_bytes(self, data: bytes, tag: Optional[str] = None) -> List[bytes]:
        """Every rank's ``data`` (raw bytes), in rank order."""
        t = self._tag(tag)
        self._write(f"{t}.{self.rank}", bytes(data))
        return [self._wait(f"{t}.{r}") for r in range(self.world)]

    def broadcast_bytes(self, data: Optional[bytes], src: int = 0, tag: Optional[str] = None) -> bytes:
        t = self._tag(tag)
        if self.rank == src:
            if data is None:
                raise ValueError("the source rank must pass the bytes")
            self._write(f"{t}.bcast", data)
            return data
        return self._wait(f"{t}.bcast")

    def barrier(self, tag: Optional[str] = None) -> None:
        self.allgather(None, tag or "barrier")

    def max(self, v: float, tag: Optional[str] = None) -> float:
        return max(float(x) for x in self.allgather(float(v), tag or "max"))

    def sum(self, v: float, tag: Optional[str] = None) -> float:
        """Sum in rank order (a fixed order: every rank gets the same bits)."""
        s = 0.0
        for x in self.allgather(float(v), tag or "sum"):
            s += float(x)
        return s

    def close(self) -> None:
        """Last barrier; then every rank reports that it has stopped reading,
        and rank 0 removes a directory it did not get from ``spawn``."""
        self.barrier("close")
        self._write(f"done.{self.rank}", b"")
        if self.rank == 0:
            for r in range(self.world):
                self._wait(f"done.{r}")
            if not os.environ.get("ZF_RDZV_DIR"):
                shutil.rmtree(self.path, ignore_errors=True)


def _start_time(pid: int) -> str:
    """Start time (clock ticks since boot) of ``pid``: with the pid it names
    one process uniquely, so a reused pid cannot meet a stale directory."""
    try:
        stat = Path(f"/proc/{pid}/stat").read_text()
        return stat.rsplit(")", 1)[1].split()[19]
    except (OSError, IndexError):
        return "0"
