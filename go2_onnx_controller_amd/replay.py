"""ObservationAction log replay.

The reference controller publishes one `onnx_interfaces/msg/ObservationAction`
per tick on `/observation_action` (controller.cpp:225-229; the message is
`float32[98] observation`, `float32[12] action`,
onnx_interfaces/msg/ObservationAction.msg:1-2): the observation it fed to
`act()` and the action after post-processing (clamp +-kActionLimit, stop
button zeroing, controller.cpp:217-223). `ros2 bag record /observation_action`
stores those messages in a rosbag2 sqlite3 database (.db3): tables `topics`
(id, name, type, serialization_format, ...) and `messages` (id, topic_id,
timestamp, data), each `data` one CDR-serialized message: a 4-byte
encapsulation header (0x00 0x01 = CDR little endian, 2 option bytes) followed
by the two fixed-size float32 arrays (no length prefix for fixed arrays).

This module reads such a bag (or an .npz with `observation`, `action`
arrays), replays the logged observations through the engine in one batched
launch (rows are independent: the history is inside each observation), and
compares against the logged actions — parity on real robot data. It also
checks the log's own consistency: tick t's history blocks must hold tick
t-1's newest values (populate_buffer, controller.hpp:45-68), in particular
the previous-action block must equal the previous logged action.
"""
from __future__ import annotations

import os
import sqlite3
from dataclasses import dataclass

import numpy as np

MSG_TYPE = "onnx_interfaces/msg/ObservationAction"
TOPIC = "/observation_action"
OBS_DIM, ACT_DIM = 98, 12
CDR_LE = b"\x00\x01\x00\x00"
# (width) of the observation's history blocks, controller.cpp:210-212
BLOCK_DIMS = (3, 3, 3, 12, 12, 12, 4)


@dataclass
class ObservationActionLog:
    t_ns: np.ndarray         # [N] int64 receive timestamps (bag) or tick index (npz without t)
    observation: np.ndarray  # [N, obs_dim] float32
    action: np.ndarray       # [N, 12] float32


def encode_cdr(obs: np.ndarray, act: np.ndarray) -> bytes:
    """One ObservationAction message, CDR little endian (as rclcpp serializes it)."""
    o = np.asarray(obs, "<f4").reshape(-1)
    a = np.asarray(act, "<f4").reshape(-1)
    return CDR_LE + o.tobytes() + a.tobytes()


def decode_cdr(data: bytes, obs_dim: int = OBS_DIM, act_dim: int = ACT_DIM):
    """Inverse of encode_cdr; accepts big-endian CDR (0x00 0x00) too."""
    if len(data) < 4:
        raise ValueError("CDR message shorter than its encapsulation header")
    kind = data[1]
    if data[0] != 0 or kind not in (0, 1):
        raise ValueError(f"unsupported CDR encapsulation {data[:2].hex()}")
    need = 4 + 4 * (obs_dim + act_dim)
    if len(data) < need:
        raise ValueError(f"ObservationAction payload has {len(data)} bytes, needs {need}")
    dt = "<f4" if kind == 1 else ">f4"
    obs = np.frombuffer(data, dt, obs_dim, 4).astype(np.float32)
    act = np.frombuffer(data, dt, act_dim, 4 + 4 * obs_dim).astype(np.float32)
    return obs, act


def _db3_path(path: str) -> str:
    if os.path.isdir(path):  # a bag directory: metadata.yaml + <name>_0.db3
        dbs = sorted(f for f in os.listdir(path) if f.endswith(".db3"))
        if not dbs:
            raise FileNotFoundError(f"no .db3 file in bag directory {path}")
        return os.path.join(path, dbs[0])
    return path


def read_bag(path: str, topic: str | None = None, obs_dim: int = OBS_DIM) -> ObservationActionLog:
    """ObservationAction messages of a rosbag2 sqlite3 bag, in timestamp order."""
    db = _db3_path(path)
    con = sqlite3.connect(f"file:{db}?mode=ro", uri=True)
    try:
        rows = con.execute("SELECT id, name, type, serialization_format FROM topics").fetchall()
        cand = [r for r in rows if r[2] == MSG_TYPE and (topic is None or r[1] == topic)]
        if not cand:
            raise ValueError(f"no {MSG_TYPE} topic in {db} (topics: {[r[1] for r in rows]})")
        tid, _, _, fmt = cand[0]
        if fmt != "cdr":
            raise ValueError(f"unsupported serialization format {fmt!r}")
        msgs = con.execute("SELECT timestamp, data FROM messages WHERE topic_id = ? ORDER BY timestamp, id",
                           (tid,)).fetchall()
    finally:
        con.close()
    n = len(msgs)
    t = np.empty(n, np.int64)
    obs = np.empty((n, obs_dim), np.float32)
    act = np.empty((n, ACT_DIM), np.float32)
    for i, (ts, data) in enumerate(msgs):
        t[i] = ts
        obs[i], act[i] = decode_cdr(bytes(data), obs_dim)
    return ObservationActionLog(t, obs, act)


def write_bag(path: str, log: ObservationActionLog, topic: str = TOPIC, distro: str = "humble") -> str:
    """Write a rosbag2 sqlite3 bag directory (metadata.yaml + <dir>_0.db3) holding `log`."""
    os.makedirs(path, exist_ok=True)
    name = os.path.basename(os.path.normpath(path))
    db = os.path.join(path, f"{name}_0.db3")
    if os.path.exists(db):
        os.remove(db)
    con = sqlite3.connect(db)
    try:
        con.execute("CREATE TABLE schema(schema_version INTEGER PRIMARY KEY, ros_distro TEXT NOT NULL)")
        con.execute("INSERT INTO schema VALUES (3, ?)", (distro,))
        con.execute("CREATE TABLE topics(id INTEGER PRIMARY KEY, name TEXT NOT NULL, type TEXT NOT NULL, "
                    "serialization_format TEXT NOT NULL, offered_qos_profiles TEXT NOT NULL)")
        con.execute("CREATE TABLE messages(id INTEGER PRIMARY KEY, topic_id INTEGER NOT NULL, "
                    "timestamp INTEGER NOT NULL, data BLOB NOT NULL)")
        con.execute("CREATE INDEX timestamp_idx ON messages (timestamp ASC)")
        con.execute("INSERT INTO topics VALUES (1, ?, ?, 'cdr', '')", (topic, MSG_TYPE))
        con.executemany("INSERT INTO messages (topic_id, timestamp, data) VALUES (1, ?, ?)",
                        [(int(t), encode_cdr(o, a)) for t, o, a in zip(log.t_ns, log.observation, log.action)])
        con.commit()
    finally:
        con.close()
    n = len(log.t_ns)
    t0 = int(log.t_ns[0]) if n else 0
    dur = int(log.t_ns[-1] - log.t_ns[0]) if n else 0
    with open(os.path.join(path, "metadata.yaml"), "w") as fh:
        fh.write("rosbag2_bagfile_information:\n  version: 5\n  storage_identifier: sqlite3\n"
                 f"  duration:\n    nanoseconds: {dur}\n  starting_time:\n    nanoseconds_since_epoch: {t0}\n"
                 f"  message_count: {n}\n  topics_with_message_count:\n    - topic_metadata:\n"
                 f"        name: {topic}\n        type: {MSG_TYPE}\n        serialization_format: cdr\n"
                 f"        offered_qos_profiles: ''\n      message_count: {n}\n"
                 f"  compression_format: ''\n  compression_mode: ''\n  relative_file_paths:\n    - {name}_0.db3\n")
    return path


def read_log(path: str) -> ObservationActionLog:
    """A bag (directory or .db3) or an .npz with `observation` / `action` (+ optional `t_ns`)."""
    if path.endswith(".npz"):
        z = np.load(path)  # allow_pickle=False: data only
        obs = np.asarray(z["observation"], np.float32)
        t = np.asarray(z["t_ns"], np.int64) if "t_ns" in z.files else np.arange(len(obs), dtype=np.int64)
        return ObservationActionLog(t, obs, np.asarray(z["action"], np.float32))
    return read_bag(path)


def history_breaks(log: ObservationActionLog, history: int | None = None) -> np.ndarray:
    """Indices t >= 1 where tick t's observation is not tick t-1's shifted by one
    step (a dropped message, a controller restart, or a corrupt log): every
    history block's older slots must equal tick t-1's newer slots, and the
    newest previous-action slot must equal action[t-1]."""
    obs, act = log.observation, log.action
    H = history or obs.shape[1] // 49
    bad = np.zeros(len(obs), bool)
    if len(obs) < 2 or H < 1:
        return np.nonzero(bad)[0]
    prev, cur = obs[:-1], obs[1:]
    ok = np.ones(len(cur), bool)
    cum = 0
    for bi, d in enumerate(BLOCK_DIMS):
        s = H * cum
        ok &= np.all(cur[:, s:s + (H - 1) * d] == prev[:, s + d:s + H * d], axis=1)
        if bi == 5:  # newest previous-action slot = the action logged at t-1
            n0 = s + (H - 1) * d
            ok &= np.all(cur[:, n0:n0 + d] == act[:-1], axis=1)
        cum += d
    bad[1:] = ~ok
    return np.nonzero(bad)[0]


def post_process(y: np.ndarray, limit: float = 1000.0) -> np.ndarray:
    """The clamp the logged action went through (controller.cpp:217-220)."""
    lim = np.float32(limit)
    y = np.asarray(y, np.float32)
    return np.where(y < -lim, -lim, np.where(lim < y, lim, y)).astype(np.float32)


@dataclass
class ReplayResult:
    n: int
    stopped: np.ndarray      # ticks whose logged action is all zero (stop button held)
    max_abs_err: float       # over the other ticks
    max_rel_err: float       # |d| / max(1, |logged|)
    worst_tick: int
    history_breaks: np.ndarray


def replay(engine, log: ObservationActionLog, limit: float = 1000.0) -> ReplayResult:
    """Run every logged observation through `engine` (one batched launch per
    engine.max_batch rows) and compare with the logged actions."""
    obs, act = log.observation, log.action
    n = len(obs)
    y = np.empty((n, engine.out_dim), np.float32)
    for i in range(0, n, engine.max_batch):
        y[i:i + engine.max_batch] = engine.run(obs[i:i + engine.max_batch])
    a = post_process(y, limit)
    stopped = np.all(act == 0, axis=1) & np.any(a != 0, axis=1)
    keep = ~stopped
    d = np.abs(a.astype(np.float64) - act)
    rel = d / np.maximum(1.0, np.abs(act.astype(np.float64)))
    d[~keep] = 0
    rel[~keep] = 0
    worst = int(np.argmax(rel.max(axis=1))) if n else -1
    return ReplayResult(n, np.nonzero(stopped)[0], float(d.max()) if n else 0.0, float(rel.max()) if n else 0.0,
                        worst, history_breaks(log))



def main(argv=None):
    """python -m go2_onnx_controller_amd.replay <bag dir | .db3 | .npz> [--model policy.onnx]"""
    import argparse
    import json
    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("log")
    ap.add_argument("--model", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                    "tests", "golden", "model.onnx"))
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--action-limit", type=float, default=1000.0)
    args = ap.parse_args(argv)
    from .engine import Engine
    log = read_log(args.log)
    with Engine(args.model, device=args.device, max_batch=max(8, min(len(log.t_ns), 65536))) as e:
        r = replay(e, log, args.action_limit)
    print(json.dumps({"ticks": r.n, "max_abs_err": r.max_abs_err, "max_rel_err": r.max_rel_err,
                      "worst_tick": r.worst_tick, "stopped_ticks": r.stopped.tolist(),
                      "history_breaks": r.history_breaks.tolist()}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
