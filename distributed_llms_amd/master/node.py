"""Master node: worker registry, heartbeat eviction, stage planning, request routing.

Reference: ``src/master/node.py`` (ROUTER socket that connects instead of binding (D1),
static-called protocol methods (D2), registry mutated from per-message threads without
locks (D21), round-robin interleaved shard assignment (D12), tokenizer input that can
never be encoded (D8), a busy-polled shared result queue (D17), ``last_heartbeat``
written but never read (D15)).  Same API, redesigned:

* binds a TCP listener; one reader thread per worker connection; all registry state under
  one lock; per-request futures (no polling);
* ``initialize_model`` shards a local HF checkpoint into the reference's ``shards/`` layout
  (contiguous, cost-balanced ranges) or selects a ``synthetic:<preset>`` random-init model
  that every worker generates on its own device (no bytes on the wire);
* ``assign_shards`` maps shard i -> i-th worker (pipeline stage i), HBM-capacity checked;
* ``distribute_shards`` sends each worker its plan (layer range, shard path, engine config,
  torch.distributed rendezvous); workers join the RCCL group and ack SHARD_LOADED;
* ``run_inference`` / ``generate`` route token ids to the stage-0 worker and wait on a future;
* a monitor thread evicts workers whose heartbeat is older than ``heartbeat_timeout``, fails
  their in-flight requests, tears the pipeline down and (``auto_recover``) re-distributes
  once enough workers are registered again.
"""
from __future__ import annotations

import concurrent.futures as cf
import itertools
import logging
import os
import queue
import socket
import threading
import time
from typing import Any, Dict, List, Optional, Sequence

from ..config import EngineConfig, ModelConfig, get_model_config
from ..network.protocol import MessageProtocol, pack_ids, unpack_ids
from ..utils.metrics import RequestMetrics
from ..utils.tokenizer import get_tokenizer

log = logging.getLogger("dllm.master")


class WorkerFailure(RuntimeError):
    pass


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class MasterNode:
    def __init__(self, host: str = "0.0.0.0", port: int = 65432, config: Optional[EngineConfig] = None,
                 auto_recover: bool = False, max_retries: Optional[int] = None):
        self.host = host
        self.port = port
        self.config = config or EngineConfig()
        self.auto_recover = auto_recover
        # in-flight requests of a failed pipeline are re-run from their prompts after recovery, at
        # most this many times each (reference intent: retry + state recovery, plan.md:430-436)
        self.max_retries = (3 if auto_recover else 0) if max_retries is None else max_retries
        self.workers: Dict[str, Dict[str, Any]] = {}
        self.model_path: Optional[str] = None
        self.model_spec: Optional[str] = None
        self.model_config: Optional[ModelConfig] = None
        self.tokenizer = None
        self.shard_manager = None
        self.shard_assignments: Dict[str, List[int]] = {}
        self.num_shards = 0
        self.stage_workers: List[str] = []       # worker id of stage i
        self.running = False
        self.server_socket: Optional[socket.socket] = None
        self.proto = MessageProtocol()
        self.state = "idle"                       # idle | ready | degraded | failed
        self._recovering = False                  # a recovery thread is running (guarded by _lock)
        self._recovery_gen = 0                    # bumped per recovery thread: only the newest clears
        #                                           _recovering or gives up (advisor round 5)
        self.recoveries = 0                       # completed re-plans after a stage loss
        self.recover_timeout = 600.0              # seconds a recovery waits for replacement workers
        self.metrics = RequestMetrics()
        self._lock = threading.RLock()
        self._ids = itertools.count()
        self._tasks: Dict[str, cf.Future] = {}
        self._reqs: Dict[str, Dict[str, Any]] = {}       # task_id -> prompt / params / attempts (for retry)
        self._retry: List[Dict[str, Any]] = []           # requests parked while the pipeline recovers
        self.max_parked = 4096                            # bound on requests held while degraded
        self._streams: Dict[str, "queue.Queue"] = {}     # task_id -> (offset, new ids) chunks, None = done
        self._acks: Dict[str, cf.Future] = {}
        self._status_futs: Dict[str, cf.Future] = {}
        self._threads: List[threading.Thread] = []
        self._registered = threading.Condition(self._lock)

    # ---------------------------------------------------------------- lifecycle
    def start(self):
        self.server_socket = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.server_socket.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.server_socket.bind((self.host, self.port))     # bind, never connect (D1)
        self.server_socket.listen(64)
        self.port = self.server_socket.getsockname()[1]
        self.running = True
        for fn in (self._accept_connections, self._monitor):
            th = threading.Thread(target=fn, daemon=True)
            th.start()
            self._threads.append(th)
        log.info("master listening on %s:%d", self.host, self.port)
        return self

    def stop(self, shutdown_workers: bool = True):
        if shutdown_workers:
            with self._lock:
                socks = [w["socket"] for w in self.workers.values()]
            for s in socks:
                self.proto.send_message(s, "SHUTDOWN")
        self.running = False
        try:
            if self.server_socket:
                self.server_socket.close()
        except OSError:
            pass
        with self._lock:
            for w in self.workers.values():
                try:
                    w["socket"].close()
                except OSError:
                    pass
            self._fail_all(WorkerFailure("master stopped"))

    # ---------------------------------------------------------------- registry
    def _accept_connections(self):
        while self.running:
            try:
                c, addr = self.server_socket.accept()
            except OSError:
                break
            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            th = threading.Thread(target=self._handle_worker, args=(c, addr), daemon=True)
            th.start()

    def _handle_worker(self, sock: socket.socket, address):
        worker_id = None
        try:
            header, _ = self.proto.receive_message(sock, timeout=30)
            if header.get("command") != "REGISTER":
                raise ValueError(f"first message must be REGISTER, got {header.get('command')}")
            worker_id = f"w{next(self._ids)}"
            with self._lock:
                self.workers[worker_id] = {
                    "worker_id": worker_id, "socket": sock, "address": f"{address[0]}:{address[1]}",
                    "connected_time": time.time(), "last_heartbeat": time.time(), "status": "connected",
                    "capabilities": header.get("capabilities", {}),
                }
                self._registered.notify_all()
            self.proto.send_message(sock, "REGISTER_ACK", metadata={
                "worker_id": worker_id, "heartbeat_interval": self.config.heartbeat_interval})
            log.info("worker %s registered from %s: %s", worker_id, address, header.get("capabilities"))
            while self.running:
                try:
                    header, payload = self.proto.receive_message(sock, timeout=None)
                except TimeoutError:
                    continue
                if not header:
                    break
                self._handle_worker_command(worker_id, header.get("command", ""), header, payload)
        except (OSError, ConnectionError, ValueError, TimeoutError) as e:
            if self.running:
                log.warning("worker %s connection error: %s", worker_id or address, e)
        finally:
            if worker_id is not None:
                self._evict(worker_id, "disconnected")

    def _handle_worker_command(self, worker_id: str, command: str, header: Dict[str, Any], payload):
        if command == "HEARTBEAT":
            with self._lock:
                w = self.workers.get(worker_id)
                if w:
                    w["last_heartbeat"] = time.time()
                    w["load"] = {k: header[k] for k in ("running", "waiting", "steps") if k in header}
        elif command == "SHARD_LOADED":
            fut = self._acks.get(worker_id)
            with self._lock:
                if worker_id in self.workers:
                    self.workers[worker_id]["shard_info"] = header
                    self.workers[worker_id]["status"] = "loaded"
            if fut and not fut.done():
                fut.set_result(header)
        elif command == "TOKENS":
            q = self._streams.get(header.get("task_id"))
            if q is not None:
                q.put((int(header.get("offset", 0)), unpack_ids(payload)))
        elif command == "RESULT":
            with self._lock:
                fut = self._tasks.pop(header.get("task_id"), None)
                self._reqs.pop(header.get("task_id"), None)
            if fut and not fut.done():
                fut.set_result((header, unpack_ids(payload)))
            q = self._streams.get(header.get("task_id"))
            if q is not None:
                q.put(None)                         # the stream's end: the full ids are in the future
        elif command == "STATUS_REPLY":
            fut = self._status_futs.pop(header.get("req"), None)
            if fut and not fut.done():
                fut.set_result(header.get("status"))
        elif command == "ERROR":
            log.error("worker %s error: %s", worker_id, header.get("error"))
            with self._lock:
                fut = self._tasks.pop(header.get("task_id"), None) if header.get("task_id") else None
                self._reqs.pop(header.get("task_id"), None)
            if fut and not fut.done():
                fut.set_exception(RuntimeError(header.get("error")))
            ack = self._acks.get(worker_id)
            if header.get("failed_command") == "LOAD_SHARD" and ack and not ack.done():
                ack.set_exception(RuntimeError(f"{worker_id} failed to load its shard: {header.get('error')}"))
        elif command == "SHARD_UNLOADED":
            with self._lock:
                if worker_id in self.workers:
                    self.workers[worker_id]["status"] = "connected"

    def _evict(self, worker_id: str, reason: str):
        with self._lock:
            w = self.workers.pop(worker_id, None)
            if w is None:
                return
            try:
                w["socket"].close()
            except OSError:
                pass
            log.warning("worker %s evicted (%s)", worker_id, reason)
            in_plan = worker_id in self.stage_workers
            ack = self._acks.get(worker_id)
            if ack and not ack.done():
                ack.set_exception(WorkerFailure(f"{worker_id} {reason}"))
            if in_plan and self.state == "ready":
                self.state = "degraded"
                exc = WorkerFailure(f"pipeline stage worker {worker_id} {reason}")
                if self.auto_recover and self.max_retries > 0:
                    self._park_inflight(exc)
                else:
                    self._fail_all(exc)
                # tear the surviving stages down: their RCCL group lost a member
                for wid in self.stage_workers:
                    ww = self.workers.get(wid)
                    if ww:
                        self.proto.send_message(ww["socket"], "UNLOAD_SHARD", metadata={"pipeline": True})
                if self.auto_recover:
                    self._recovering = True
                    self._recovery_gen += 1
                    threading.Thread(target=self._recover_when_possible, kwargs={"gen": self._recovery_gen},
                                     daemon=True).start()

    def _fail_all(self, exc: Exception):
        with self._lock:
            tasks, self._tasks = self._tasks, {}
            self._reqs.clear()
            parked, self._retry = self._retry, []
            streams = list(self._streams.values())
        for fut in list(tasks.values()) + [r["future"] for r in parked]:
            if not fut.done():
                fut.set_exception(exc)
        # streams end (their futures carry the error) -- the parked ones too: their queues left
        # self._streams when they were parked
        for q in streams + [r["stream"] for r in parked if r.get("stream") is not None]:
            q.put(None)

    def _park_inflight(self, exc: Exception):
        """The pipeline lost a stage: keep every in-flight request's future pending and park it
        for re-submission once the pipeline is back.  Fail now: requests out of retries, and
        SAMPLED streaming requests -- a re-run from the prompt draws different tokens, which the
        client would get spliced onto the prefix it already streamed (greedy re-runs reproduce the
        prefix exactly, so the stream resumes where it was)."""
        with self._lock:
            tasks, self._tasks = self._tasks, {}
            reqs, self._reqs = self._reqs, {}
            fail = []
            for tid, fut in tasks.items():
                r = reqs.get(tid)
                q = self._streams.pop(tid, None)
                if fut.done():
                    continue
                sampled = r is not None and float(r["params"].get("temperature", 0.0) or 0.0) > 0.0
                if r is None or r["attempts"] >= self.max_retries or (q is not None and sampled):
                    fail.append((fut, q))
                    continue
                r["future"] = fut
                r["stream"] = q
                self._retry.append(r)
        for fut, q in fail:
            fut.set_exception(exc)
            if q is not None:
                q.put(None)
        log.warning("%d in-flight requests parked for retry, %d failed", len(self._retry), len(fail))

    def _resubmit_parked(self):
        with self._lock:
            parked, self._retry = self._retry, []
        for r in parked:
            r["attempts"] += 1
            try:
                self._send_request(r["ids"], r["params"], r["future"], r["stream"], r["hint"], r["attempts"])
            except WorkerFailure as e:
                if not r["future"].done():
                    r["future"].set_exception(e)
                if r.get("stream") is not None:
                    r["stream"].put(None)
        if parked:
            log.info("re-submitted %d requests after recovery", len(parked))

    def _monitor(self):
        """Heartbeat-timeout eviction (the reference records last_heartbeat and never reads it, D15)."""
        while self.running:
            time.sleep(max(0.2, self.config.heartbeat_interval / 2))
            now = time.time()
            with self._lock:
                stale = [wid for wid, w in self.workers.items()
                         if now - w["last_heartbeat"] > self.config.heartbeat_timeout]
            for wid in stale:
                self._evict(wid, "heartbeat timeout")

    def wait_for_workers(self, n: int, timeout: float = 120.0) -> List[str]:
        t_end = time.time() + timeout
        with self._lock:
            while len(self.workers) < n:
                left = t_end - time.time()
                if left <= 0:
                    raise TimeoutError(f"only {len(self.workers)}/{n} workers registered")
                self._registered.wait(left)
            return sorted(self.workers, key=lambda k: int(k[1:]))

    # ---------------------------------------------------------------- model / shards
    def initialize_model(self, model_id: str, num_shards: int, cache_dir: str = "./models") -> str:
        """Checkpoint dir -> shards/ layout (contiguous ranges); ``synthetic:<preset>`` -> no files."""
        from ..checkpoint.loader import download_model, load_tokenizer
        from ..checkpoint.shard_manager import ModelShardManager
        self.num_shards = num_shards
        if model_id.startswith("synthetic:") or (model_id in __import__(
                "distributed_llms_amd.config", fromlist=["PRESETS"]).PRESETS):
            spec = model_id if model_id.startswith("synthetic:") else f"synthetic:{model_id}"
            self.model_spec = spec
            self.model_path = None
            self.model_config = get_model_config(spec)
            self.tokenizer = get_tokenizer(None, self.model_config.vocab_size)
            return spec
        self.model_path = model_id if os.path.isdir(model_id) else download_model(model_id, cache_dir)
        self.model_spec = self.model_path
        self.model_config = get_model_config(self.model_path)
        self.tokenizer = get_tokenizer(load_tokenizer(self.model_path), self.model_config.vocab_size)
        self.shard_manager = ModelShardManager(self.model_path, num_shards, self.model_config)
        return self.shard_manager.shard_model()

    def _plan_device(self) -> str:
        """The cost model the stage planner uses: "cpu" when every (stage) worker is a CPU worker."""
        with self._lock:
            ws = [self.workers[w] for w in (self.stage_workers or list(self.workers)) if w in self.workers]
        devs = [str(w.get("capabilities", {}).get("device", "cuda")) for w in ws]
        return "cpu" if devs and all(d.startswith("cpu") for d in devs) else "cuda"

    def stage_weight_bytes(self) -> List[int]:
        """bf16/fp16 weight bytes each pipeline stage will hold (layers + embedding / LM head)."""
        from ..parallel.planner import plan_units
        cfg = self.model_config
        n = self.num_shards
        if self.shard_manager is not None:
            return [os.path.getsize(p) for p in self.shard_manager.get_shard_paths()]
        up = plan_units(cfg, n, batch=self.config.max_batch, ctx=max(32, self.config.max_seq_len // 2),
                            device=self._plan_device())
        width = 4 if self.config.dtype == "float32" else 2
        per_layer = cfg.layer_param_count() * width
        out = []
        for i, (a, b) in enumerate(up.ranges):
            nbytes = (b - a) * per_layer
            if i == 0 or i == n - 1:
                nbytes += cfg.head_param_count() * width // (1 if n == 1 else 2)
            out.append(int(nbytes))
        return out

    def assign_shards(self) -> Dict[str, List[int]]:
        """Stage i -> a registered worker, capacity-aware (SURVEY §2.8 "capacity-aware assignment").

        Candidates are the workers whose device memory can hold the stage's weights plus KV
        headroom (``memory`` from REGISTER; CPU workers report 0 and only serve CPU configs).  With
        more workers than stages the largest devices are used; stages keep registration order
        among equals so pipeline neighbours stay predictable.  The reference assigned round-robin
        and ignored capabilities (``src/master/node.py:84-104``)."""
        with self._lock:
            if not self.workers:
                raise ValueError("No workers connected")
            if not self.num_shards:
                raise ValueError("initialize_model() first")
            workers = sorted(self.workers, key=lambda k: int(k[1:]))
            if len(workers) < self.num_shards:
                raise ValueError(f"{self.num_shards} shards need {self.num_shards} workers, have {len(workers)}")
            mem = {w: int(self.workers[w].get("capabilities", {}).get("memory", 0) or 0) for w in workers}
            if any(mem.values()):
                need = self.stage_weight_bytes()
                # the largest devices first, registration order among equals
                pool = sorted(workers, key=lambda w: (-mem[w], int(w[1:])))[: self.num_shards]
                pool.sort(key=lambda w: int(w[1:]))
                order = sorted(range(self.num_shards), key=lambda i: -need[i])
                by_mem = sorted(pool, key=lambda w: (-mem[w], int(w[1:])))
                chosen = [None] * self.num_shards
                for i, w in zip(order, by_mem):       # heaviest stage -> largest device
                    if mem[w] and need[i] * 1.1 > mem[w]:
                        raise ValueError(f"stage {i} needs {need[i] / 2**30:.1f} GiB of weights; worker {w} "
                                         f"has {mem[w] / 2**30:.1f} GiB")
                    chosen[i] = w
                if sorted(mem[w] for w in pool) == [mem[pool[0]]] * len(pool):
                    chosen = pool                     # homogeneous node: keep registration order
                self.stage_workers = chosen
            else:
                self.stage_workers = workers[: self.num_shards]
            self.shard_assignments = {wid: [i] for i, wid in enumerate(self.stage_workers)}
            return dict(self.shard_assignments)

    def _plans(self) -> List[Dict[str, Any]]:
        from ..parallel.planner import plan_units
        cfg = self.model_config
        n = self.num_shards
        if self.shard_manager is not None:
            ranges = [tuple(r) for r in self.shard_manager.read_plan(self.shard_manager.shard_dir)["ranges"]]
            unit_ranges = [(2 * a, 2 * b) for a, b in ranges]
            group = 2
            paths = self.shard_manager.get_shard_paths()
        else:
            up = plan_units(cfg, n, batch=self.config.max_batch, ctx=max(32, self.config.max_seq_len // 2),
                            device=self._plan_device())
            ranges = list(up.ranges)
            unit_ranges = list(up.units)
            group = up.group
            paths = [None] * n
        ecfg = self.config.apply_overrides(model=self.model_spec, num_workers=n)
        ed = ecfg.to_dict()
        if self.shard_manager is not None:
            ed["shard_dir"] = self.shard_manager.shard_dir
        master_addr = self.config.host if self.config.host not in ("0.0.0.0", "") else "127.0.0.1"
        dist = {"master_addr": os.environ.get("DLLM_DIST_ADDR", "127.0.0.1" if master_addr == "0.0.0.0" else master_addr),
                "master_port": _free_port()}
        # stage workers sharing a host: CPU workers split its cores instead of oversubscribing them
        with self._lock:
            hosts = [(self.workers.get(w) or {}).get("capabilities", {}).get("host") for w in self.stage_workers]
        hosts += [None] * (n - len(hosts))
        host_workers = [sum(1 for h in hosts if h is not None and h == hosts[i]) or 1 for i in range(n)]
        return [{"shard_id": i, "stage": i, "num_stages": n, "layer_range": list(ranges[i]),
                 "unit_range": list(unit_ranges[i]), "unit_group": group, "host_workers": host_workers[i],
                 "shard_path": paths[i], "engine_config": ed, "dist": dist} for i in range(n)]

    def distribute_shards(self, timeout: float = 1800.0, ship_bytes: bool = False) -> Dict[str, Any]:
        """Send every stage worker its plan; wait for all SHARD_LOADED acks."""
        if not self.shard_assignments:
            self.assign_shards()
        plans = self._plans()
        futs = {}
        with self._lock:
            for i, wid in enumerate(self.stage_workers):
                w = self.workers.get(wid)
                if w is None:
                    raise WorkerFailure(f"worker {wid} is gone")
                futs[wid] = self._acks[wid] = cf.Future()
        for i, wid in enumerate(self.stage_workers):
            payload = None
            plan = plans[i]
            if ship_bytes and plan["shard_path"]:
                with open(plan["shard_path"], "rb") as f:    # cross-host: ship the file itself
                    payload = f.read()
                plan = dict(plan, shard_path=None)
            ok = self.proto.send_message(self.workers[wid]["socket"], "LOAD_SHARD", payload=payload,
                                         metadata={"plan": plan, "shard_id": i})
            if not ok:
                raise WorkerFailure(f"cannot send plan to {wid}")
        acks = {wid: f.result(timeout=timeout) for wid, f in futs.items()}
        self.state = "ready"
        log.info("pipeline ready: %s", {w: a.get("layer_range") for w, a in acks.items()})
        return acks

    def _recover_when_possible(self, timeout: Optional[float] = None, gen: Optional[int] = None):
        """Re-admit a full set of stage workers (waits for replacements), reload the plan, then
        re-run the parked requests from their prompts.  Failed attempts back off exponentially.

        ``_recovering`` is set (under the lock) by whoever starts this thread and cleared here under
        the same lock as the final hand-over: on success together with the resubmission of the
        parked requests, on give-up together with the state change to "failed" and the swap-out of
        the parked list -- so a concurrent submit() either parks before that swap (and is failed or
        resubmitted with the rest) or sees "failed" / "ready" and never parks into a list that
        nobody will drain.

        ``gen``: this thread's recovery generation.  A stage worker evicted after this thread has
        re-admitted the pipeline (e.g. while it re-submits the parked requests) starts a newer
        thread; this one then leaves ``_recovering``, the state and the newly parked requests to
        that thread instead of declaring the pipeline failed from the state it now sees."""
        t_end = time.time() + (self.recover_timeout if timeout is None else timeout)
        backoff = 0.5
        if gen is None:
            with self._lock:
                gen = self._recovery_gen
        recovered = False
        try:
            while self.running and time.time() < t_end and self.state == "degraded":
                with self._lock:
                    have = len(self.workers)
                if have >= self.num_shards:
                    try:
                        self.shard_assignments = {}
                        self.assign_shards()
                        self.distribute_shards()
                        recovered = True
                        self.recoveries += 1
                        log.info("pipeline recovered onto %s", self.stage_workers)
                        self._resubmit_parked()
                        return
                    except Exception as e:
                        log.error("recovery attempt failed: %s (next in %.1fs)", e, backoff)
                        time.sleep(backoff)
                        backoff = min(30.0, backoff * 2)
                        continue
                time.sleep(0.5)
        finally:
            with self._lock:
                newest = gen == self._recovery_gen
                gave_up = newest and not recovered
                if newest:
                    self._recovering = False
                if gave_up:
                    self.state = "failed"
            if gave_up:
                self._fail_all(WorkerFailure("pipeline did not recover"))

    # ---------------------------------------------------------------- inference
    def submit(self, prompt_ids: Sequence[int], params: Optional[Dict[str, Any]] = None, _stream_queue=None,
               _task_out=None) -> cf.Future:
        fut: cf.Future = cf.Future()
        fut.t_submit = time.perf_counter()
        ids, params = list(prompt_ids), dict(params or {})
        with self._lock:
            # degraded with recovery on: hold the request with the parked in-flight ones (bounded)
            # until the stage is re-admitted (plan.md:430-436) -- checked under the
            # lock that _resubmit_parked takes after the state is back to "ready", so a request
            # is either parked before the resubmission or sent directly after it
            if self.state == "degraded" and self.auto_recover and self._recovering and self.running:
                if len(self._retry) >= self.max_parked:
                    raise WorkerFailure(f"pipeline degraded and {len(self._retry)} requests already held")
                self._retry.append({"ids": ids, "params": params, "attempts": 0, "hint": _task_out,
                                    "future": fut, "stream": _stream_queue})
                return fut
            if self.state != "ready":
                raise WorkerFailure(f"pipeline not ready (state={self.state})")
        self._send_request(ids, params, fut, _stream_queue, _task_out, 0)
        return fut

    def _send_request(self, ids: List[int], params: Dict[str, Any], fut: cf.Future, stream_q, hint, attempts: int):
        """Register ``fut`` under a fresh task id and send the prompt to stage 0 (first try or a
        retry after recovery: a retry streams from offset 0 again and the stream consumer skips
        what it already yielded)."""
        task_id = f"task_{next(self._ids)}_{int(time.time() * 1000)}"
        fut.task_id = task_id
        with self._lock:
            self._tasks[task_id] = fut
            self._reqs[task_id] = {"ids": ids, "params": params, "attempts": attempts, "hint": hint}
            if stream_q is not None:
                self._streams[task_id] = stream_q
                if hint is not None:
                    hint["task_id"] = task_id
            w0 = self.workers.get(self.stage_workers[0]) if self.stage_workers else None
        ok = w0 is not None and self.proto.send_message(w0["socket"], "RUN_INFERENCE", payload=pack_ids(ids),
                                                        metadata={"task_id": task_id, "params": params})
        if not ok:
            with self._lock:
                self._tasks.pop(task_id, None)
                self._reqs.pop(task_id, None)
                self._streams.pop(task_id, None)
            raise WorkerFailure("stage-0 worker is gone" if w0 is None else "cannot send request to stage 0")

    def stream(self, prompt_ids: Sequence[int], timeout: float = 600, **params):
        """Generate with token streaming: yields lists of new token ids as stage 0 produces them
        (TOKENS messages, one per pipeline step that advanced the request); the last chunk is what
        the final RESULT adds.  The chunks concatenate to exactly what :meth:`submit` returns."""
        q: "queue.Queue" = queue.Queue()
        # register the queue before the request can produce anything
        task_hint = {}
        fut = self.submit(prompt_ids, dict(params, stream=True), _stream_queue=q, _task_out=task_hint)
        sent = 0
        deadline = time.time() + timeout
        try:
            while True:
                try:
                    item = q.get(timeout=max(0.01, deadline - time.time()))
                except queue.Empty:
                    raise TimeoutError("stream timed out") from None
                if item is None:
                    break
                off, ids = item
                if off + len(ids) > sent:
                    new = ids[sent - off:]
                    sent += len(new)
                    yield new
            r = self._finish(fut, max(0.01, deadline - time.time()))
            if len(r["tokens"]) > sent:
                yield r["tokens"][sent:]
        finally:
            self._streams.pop(task_hint.get("task_id"), None)

    def _finish(self, fut: cf.Future, timeout: float):
        header, ids = fut.result(timeout=timeout)
        lat = time.perf_counter() - fut.t_submit
        self.metrics.record(len(ids), lat, header.get("ttft_s"))
        return {"task_id": header.get("task_id"), "tokens": ids, "finish_reason": header.get("finish_reason"),
                "latency_s": lat, "ttft_s": header.get("ttft_s")}

    def run_inference(self, input_text, timeout: float = 60, max_new_tokens: int = 32, **params) -> Dict[str, Any]:
        """Text (tokenized on the master) or token ids -> generated ids (+ detokenized text)."""
        ids = self.tokenizer.encode(input_text) if isinstance(input_text, str) else list(input_text)
        p = dict(params, max_new_tokens=max_new_tokens)
        res = self._finish(self.submit(ids, p), timeout)
        res["text"] = self.tokenizer.decode(res["tokens"])
        return res

    def generate(self, prompts: Sequence[Sequence[int]], timeout: float = 600, **params) -> List[Dict[str, Any]]:
        futs = [self.submit(list(p), params) for p in prompts]
        return [self._finish(f, timeout) for f in futs]

    def status(self, timeout: float = 10.0) -> Dict[str, Any]:
        with self._lock:
            reg = {wid: {k: v for k, v in w.items() if k != "socket"} for wid, w in self.workers.items()}
            socks = {wid: w["socket"] for wid, w in self.workers.items()}
        futs = {}
        for wid, s in socks.items():
            req = f"st{next(self._ids)}"
            futs[wid] = self._status_futs[req] = cf.Future()
            self.proto.send_message(s, "STATUS", metadata={"req": req})
        for wid, f in futs.items():
            try:
                reg[wid]["remote"] = f.result(timeout=timeout)
            except Exception as e:
                reg[wid]["remote"] = {"error": repr(e)}
        spares = sorted(w for w in reg if w not in self.stage_workers)
        return {"state": self.state, "model": self.model_spec, "num_shards": self.num_shards,
                "stage_workers": self.stage_workers, "spare_workers": spares, "workers": reg,
                "metrics": self.metrics.summary(), "pending_requests": len(self._tasks),
                "recoveries": self.recoveries}
