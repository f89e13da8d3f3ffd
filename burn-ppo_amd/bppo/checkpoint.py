"""Checkpoint interop: the reference's checkpoint directory layout and files
(checkpoint.rs) written from / read into a device-resident context.

  checkpoints/step_%08d/{model.mpk, optimizer.mpk, metadata.json,
                         normalizer.json, return_normalizer.json, rng_state.bin}
  checkpoints/latest, checkpoints/best      relative symlinks, renamed atomically

  CheckpointMetadata                checkpoint.rs:26-96 (field names, order, serde defaults)
  CheckpointManager.save / load     checkpoint.rs:147-272 (temp dir + rename; best by avg_return)
  save/load_optimizer               checkpoint.rs:291-335
  save/load_normalizer              checkpoint.rs:340-375 (ObsNormalizer JSON)
  save/load_return_normalizer       checkpoint.rs:430-465
  save/load_popart_normalizer       checkpoint.rs:468-490
  save_rng_state / load_rng_state   checkpoint.rs:380-426: 32 bytes drawn from the
                                    main RNG (advances it by 8 words, as the reference
                                    does at every periodic checkpoint, main.rs:1307);
                                    resume = StdRng::from_seed(those bytes)

JSON: serde_json::to_string_pretty layout (2-space indent, one array element per
line) with floats in ryu's shortest form (f32 fields as f32, f64 as f64; non-finite
as null).  model.mpk / optimizer.mpk: MessagePack of Burn's NamedMpkFileRecorder
<FullPrecisionSettings> record — BurnRecord {metadata, item} with the module
record's field names (mlp.rs:47-62, ctde.rs:26-44, network/mod.rs:28-35) and
Param {id, param: TensorData {bytes, shape, dtype}}.  Burn 0.20 is not vendored
in the reference, so the byte layout of the .mpk files is restated and PARITY
UNPINNED; the JSON files and rng_state.bin follow the reference's own serde /
fs::write code exactly.
"""
import ctypes as C
import hashlib
import json
import math
import os
import shutil
from dataclasses import dataclass, field, fields
from typing import List, Optional, Tuple

import msgpack
import numpy as np

from . import _lib as L
from .host import layer_shapes

# ------------------------------------------------------------------ JSON ---


def _ryu(v, f32):
    """serde_json float text: ryu shortest digits, ryu's layout rules
    (decimal for 10^-5 <= |v| < 10^16, else d.ddde<exp>)."""
    if not math.isfinite(v):
        return "null"
    if v == 0.0:
        return "-0.0" if math.copysign(1.0, v) < 0 else "0.0"
    s = np.format_float_scientific(np.float32(v) if f32 else np.float64(v), unique=True, trim="-")
    sign = "-" if s.startswith("-") else ""
    mant, exp = s.lstrip("-").split("e")
    digits = mant.replace(".", "")
    k = int(exp) - (len(digits) - 1)          # value = digits * 10^k
    n = len(digits)
    kk = n + k                                 # 10^(kk-1) <= v < 10^kk
    if 0 <= k and kk <= 16:
        return sign + digits + "0" * k + ".0"
    if 0 < kk <= 16:
        return sign + digits[:kk] + "." + digits[kk:]
    if -5 < kk <= 0:
        return sign + "0." + "0" * (-kk) + digits
    e = str(kk - 1)
    if n == 1:
        return sign + digits + "e" + e
    return sign + digits[0] + "." + digits[1:] + "e" + e


class F32(float):
    """a float serialized as f32 (the reference's f32 fields)"""


def to_json_pretty(v, ind=""):
    """serde_json::to_string_pretty"""
    nxt = ind + "  "
    if isinstance(v, dict):
        if not v:
            return "{}"
        return "{\n" + ",\n".join(f"{nxt}{json.dumps(k)}: {to_json_pretty(x, nxt)}" for k, x in v.items()) + \
            "\n" + ind + "}"
    if isinstance(v, (list, tuple)):
        if not v:
            return "[]"
        return "[\n" + ",\n".join(nxt + to_json_pretty(x, nxt) for x in v) + "\n" + ind + "]"
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if isinstance(v, (float, np.floating)):
        return _ryu(float(v), isinstance(v, (F32, np.float32)))
    if isinstance(v, str):
        return json.dumps(v, ensure_ascii=False)
    raise TypeError(type(v))


# -------------------------------------------------------------- metadata ---
_REQUIRED = ("step", "avg_return", "rng_seed", "obs_dim", "action_count", "num_players", "hidden_size",
             "num_hidden", "activation", "env_name")


@dataclass
class CheckpointMetadata:
    """checkpoint.rs:26-96, same fields in the same order; serde defaults for the
    #[serde(default)] ones, the rest required (a file without them fails to load)."""
    step: int
    avg_return: float
    rng_seed: int
    best_avg_return: Optional[float] = None
    recent_returns: List[float] = field(default_factory=list)
    forked_from: Optional[str] = None
    obs_dim: int = 0
    action_count: int = 0
    num_players: int = 1
    hidden_size: int = 64
    num_hidden: int = 2
    activation: str = "tanh"
    split_networks: bool = False
    network_type: str = "mlp"
    num_conv_layers: int = 2
    conv_channels: List[int] = field(default_factory=lambda: [64, 64])
    kernel_size: int = 3
    cnn_fc_hidden_size: int = 128
    cnn_num_fc_layers: int = 1
    privileged_obs_dim: Optional[int] = None
    critic_hidden_size: Optional[int] = None
    critic_num_hidden: Optional[int] = None
    obs_shape: Optional[Tuple[int, int, int]] = None
    env_name: str = "cartpole"
    exploitability_vs_pool: Optional[float] = None

    _F32 = ("avg_return", "best_avg_return", "exploitability_vs_pool")

    def to_json(self):
        d = {}
        for f in fields(self):
            v = getattr(self, f.name)
            if f.name in self._F32 and v is not None:
                v = F32(v)
            elif f.name == "recent_returns":
                v = [F32(x) for x in v]
            elif f.name == "obs_shape" and v is not None:
                v = list(v)
            d[f.name] = v
        return to_json_pretty(d)

    @classmethod
    def from_json(cls, text):
        d = json.loads(text)
        if "global_state_dim" in d and "privileged_obs_dim" not in d:   # #[serde(alias)]
            d["privileged_obs_dim"] = d.pop("global_state_dim")
        missing = [k for k in _REQUIRED if k not in d]
        if missing:
            raise ValueError(f"Failed to parse checkpoint metadata (missing required fields: {missing})")
        known = {f.name for f in fields(cls)}
        m = cls(**{k: v for k, v in d.items() if k in known})
        if m.obs_shape is not None:
            m.obs_shape = tuple(m.obs_shape)
        return m

    @classmethod
    def for_config(cls, cfg, step, avg_return, recent_returns=(), best_avg_return=None, forked_from=None):
        """the metadata run_training writes (main.rs:451-476, 1245-1271): every CNN field,
        split_networks and the critic sizes straight from the config whatever the network
        type, obs_shape = E::OBSERVATION_SHAPE (Connect Four only, connect_four.rs:217),
        privileged_obs_dim for CTDE only (main.rs:215-230)"""
        from .host import ENV_DIMS
        obs, act, P, priv = ENV_DIMS[cfg["env"]]
        ctde = cfg["network_type"] == "ctde"
        return cls(step=int(step), avg_return=float(avg_return), rng_seed=int(cfg["seed"]),
                   best_avg_return=best_avg_return, recent_returns=[float(x) for x in recent_returns],
                   forked_from=forked_from, obs_dim=obs, action_count=act, num_players=P,
                   hidden_size=cfg["hidden_size"], num_hidden=cfg["num_hidden"], activation=cfg["activation"],
                   split_networks=bool(cfg.get("split_networks", False)), network_type=cfg["network_type"],
                   num_conv_layers=int(cfg["num_conv_layers"]), conv_channels=[int(c) for c in cfg["conv_channels"]],
                   kernel_size=int(cfg["kernel_size"]), cnn_fc_hidden_size=int(cfg["cnn_fc_hidden_size"]),
                   cnn_num_fc_layers=int(cfg["cnn_num_fc_layers"]), privileged_obs_dim=priv if ctde else None,
                   critic_hidden_size=cfg.get("critic_hidden_size"), critic_num_hidden=cfg.get("critic_num_hidden"),
                   obs_shape=(6, 7, 2) if cfg["env"] == "connect_four" else None, env_name=cfg["env"])


def load_metadata(ckpt_dir):
    """checkpoint.rs:279-285"""
    with open(os.path.join(ckpt_dir, "metadata.json")) as f:
        return CheckpointMetadata.from_json(f.read())


# ----------------------------------------------------------- model record ---
BURN_METADATA = {"float": "f32", "int": "i32", "format": "burn::record::file::NamedMpkFileRecorder",
                 "version": "0.20.0", "settings": "burn::record::settings::FullPrecisionSettings"}


def _param_id(path):
    return str(int.from_bytes(hashlib.sha256(path.encode()).digest()[:8], "little") >> 16)


def _tensor(a):
    a = np.ascontiguousarray(a, np.float32)
    return {"bytes": a.tobytes(), "shape": list(a.shape), "dtype": "F32"}


def _linear(W, b, path):
    return {"weight": {"id": _param_id(path + ".weight"), "param": _tensor(W)},
            "bias": {"id": _param_id(path + ".bias"), "param": _tensor(b)}}


def _split(cfg, params):
    """flat Burn-order params -> [(W [in, out], b [out])] in record order"""
    shapes, _ = layer_shapes(cfg)
    out, off = [], 0
    for i, o in shapes:
        W = params[off:off + i * o].reshape(i, o); off += i * o
        b = params[off:off + o]; off += o
        out.append((W, b))
    assert off == params.size, (off, params.size)
    return out


def model_record(cfg, params):
    """ActorCriticNetwork record item (enum variant -> {"Mlp"|"Ctde": {...}})"""
    lin = _split(cfg, np.asarray(params, np.float32))
    nh = cfg["num_hidden"]
    if cfg["network_type"] == "cnn":
        # cnn.rs:24-50: Conv2d {weight [Cout][Cin][k][k], bias}, then Linear layers
        from .host import conv_channels
        ch, ks = conv_channels(cfg), cfg["kernel_size"]
        nc, nf = len(ch), cfg["cnn_num_fc_layers"]

        def convs(lins, name):
            out = []
            for i, (W, b) in enumerate(lins):
                cin = W.shape[0] // (ks * ks)
                out.append({"weight": {"id": _param_id(f"{name}.{i}.weight"),
                                       "param": _tensor(W.reshape(-1).reshape(ch[i], cin, ks, ks))},
                            "bias": {"id": _param_id(f"{name}.{i}.bias"), "param": _tensor(b)}})
            return out
        # record order (cnn.rs:24-50): conv, fc, critic conv, critic fc (split_networks), heads
        t = nc + nf if cfg.get("split_networks") else 0
        item = {"Cnn": {"conv_layers": convs(lin[:nc], "conv_layers"),
                        "fc_layers": [_linear(W, b, f"fc_layers.{i}") for i, (W, b) in enumerate(lin[nc:nc + nf])],
                        "critic_conv_layers": convs(lin[nc + nf:nc + nf + nc], "critic_conv_layers") if t else [],
                        "critic_fc_layers": [_linear(W, b, f"critic_fc_layers.{i}")
                                             for i, (W, b) in enumerate(lin[2 * nc + nf:nc + nf + t])] if t else [],
                        "policy_head": _linear(*lin[nc + nf + t], "policy_head"),
                        "value_head": _linear(*lin[nc + nf + t + 1], "value_head")}}
        return {"metadata": BURN_METADATA, "item": item}
    if cfg["network_type"] == "ctde":
        nc = cfg["critic_num_hidden"] or nh
        item = {"Ctde": {"actor_layers": [_linear(W, b, f"actor_layers.{i}") for i, (W, b) in enumerate(lin[:nh])],
                         "policy_head": _linear(*lin[nh], "policy_head"),
                         "critic_layers": [_linear(W, b, f"critic_layers.{i}")
                                           for i, (W, b) in enumerate(lin[nh + 1:nh + 1 + nc])],
                         "value_head": _linear(*lin[nh + 1 + nc], "value_head")}}
    else:
        nc = nh if cfg.get("split_networks") else 0                     # mlp.rs:47-62 critic_layers
        item = {"Mlp": {"layers": [_linear(W, b, f"layers.{i}") for i, (W, b) in enumerate(lin[:nh])],
                        "critic_layers": [_linear(W, b, f"critic_layers.{i}")
                                          for i, (W, b) in enumerate(lin[nh:nh + nc])],
                        "policy_head": _linear(*lin[nh + nc], "policy_head"),
                        "value_head": _linear(*lin[nh + nc + 1], "value_head")}}
    return {"metadata": BURN_METADATA, "item": item}


def _linears_in_order(item):
    (kind, rec), = item.items()
    if kind == "Cnn":      # record order: conv, fc, critic conv, critic fc (split_networks), heads
        return (rec["conv_layers"] + rec["fc_layers"] + rec["critic_conv_layers"] + rec["critic_fc_layers"] +
                [rec["policy_head"], rec["value_head"]])
    if kind == "Ctde":
        seq = rec["actor_layers"] + [rec["policy_head"]] + rec["critic_layers"] + [rec["value_head"]]
    elif kind == "Mlp":      # record order: layers, critic_layers (split_networks), policy, value
        seq = rec["layers"] + rec["critic_layers"] + [rec["policy_head"], rec["value_head"]]
    else:
        raise ValueError(f"network type {kind} is not supported by the device path")
    return seq


def params_from_record(rec):
    out = []
    for lin in _linears_in_order(rec["item"]):
        for k in ("weight", "bias"):
            t = lin[k]["param"]
            out.append(np.frombuffer(t["bytes"], np.float32).reshape(t["shape"]).reshape(-1))
    return np.concatenate(out)


def save_model(cfg, params, path):
    with open(path, "wb") as f:
        f.write(msgpack.packb(model_record(cfg, params), use_bin_type=True))


def load_model(path):
    with open(path, "rb") as f:
        return params_from_record(msgpack.unpackb(f.read(), raw=False))


# ------------------------------------------------------------- optimizer ---
def optimizer_record(cfg, m1, m2, steps):
    """OptimizerAdaptor<Adam> record: per parameter id an AdamState
    {momentum: {time, moment_1, moment_2}} (burn-optim, restated)"""
    rec = model_record(cfg, np.zeros_like(m1))["item"]
    params = [lin[k] for lin in _linears_in_order(rec) for k in ("weight", "bias")]
    ids = [p["id"] for p in params]
    # each moment has its parameter's record shape (Linear [in, out] / [out]; Conv2d
    # [Cout, Cin, k, k] / [Cout]): Burn's Adam state mirrors the gradient's shape
    item, off = {}, 0
    for t, p in enumerate(params):
        shp = p["param"]["shape"]
        n = int(np.prod(shp))
        item[ids[t]] = {"momentum": {"time": int(steps[t]),
                                     "moment_1": _tensor(m1[off:off + n].reshape(shp)),
                                     "moment_2": _tensor(m2[off:off + n].reshape(shp))}}
        off += n
    assert off == m1.size, (off, m1.size)
    return {"metadata": BURN_METADATA, "item": item}, ids


def save_optimizer(ctx, path_dir):
    """checkpoint.rs:291-305 (optimizer.mpk)"""
    n = ctx.n_params
    m1 = np.zeros(n, np.float32); m2 = np.zeros(n, np.float32)
    nt = L.lib().bppo_num_param_tensors(ctx.h)
    steps = np.zeros(nt, np.int32)
    ctx._chk(L.lib().bppo_optimizer_get(ctx.h, m1.ctypes.data, m2.ctypes.data, steps.ctypes.data, n))
    rec, _ = optimizer_record(ctx.cfg, m1, m2, steps)
    with open(os.path.join(path_dir, "optimizer.mpk"), "wb") as f:
        f.write(msgpack.packb(rec, use_bin_type=True))


def model_param_ids(path_dir):
    """ParamIds of model.mpk in record order (weight, bias of each layer), or None.
    Burn keys the optimizer record by the model's ParamIds, which are random per
    model, so an optimizer.mpk is read with the ids of the model saved beside it."""
    p = os.path.join(path_dir, "model.mpk")
    if not os.path.exists(p):
        return None
    with open(p, "rb") as f:
        item = msgpack.unpackb(f.read(), raw=False)["item"]
    return [lin[k]["id"] for lin in _linears_in_order(item) for k in ("weight", "bias")]


def load_optimizer(ctx, path_dir):
    """checkpoint.rs:311-335: no optimizer.mpk -> optimizer unchanged (False)"""
    p = os.path.join(path_dir, "optimizer.mpk")
    if not os.path.exists(p):
        return False
    with open(p, "rb") as f:
        rec = msgpack.unpackb(f.read(), raw=False)
    ids = model_param_ids(path_dir)
    if ids is None:   # no model record beside it: the ids this module writes
        _, ids = optimizer_record(ctx.cfg, np.zeros(ctx.n_params, np.float32), np.zeros(ctx.n_params, np.float32),
                                  np.zeros(len(layer_shapes(ctx.cfg)[0]) * 2, np.int32))
    m1, m2, steps = optimizer_arrays(rec, ids)
    ctx._chk(L.lib().bppo_optimizer_set(ctx.h, m1.ctypes.data, m2.ctypes.data, steps.ctypes.data, ctx.n_params))
    return True


def optimizer_arrays(rec, ids):
    """flat (moment_1, moment_2, per-tensor step) of an optimizer record, tensors in
    the order of `ids` (the model's ParamIds in record order)"""
    m1, m2, steps = [], [], []
    for pid in ids:
        if pid not in rec["item"]:
            raise KeyError(f"optimizer record has no state for parameter id {pid}")
        st = rec["item"][pid]["momentum"]
        m1.append(np.frombuffer(st["moment_1"]["bytes"], np.float32))
        m2.append(np.frombuffer(st["moment_2"]["bytes"], np.float32))
        steps.append(st["time"])
    return (np.ascontiguousarray(np.concatenate(m1)), np.ascontiguousarray(np.concatenate(m2)),
            np.asarray(steps, np.int32))


# ------------------------------------------------------------ normalizers ---
def save_normalizer(ctx, path_dir, clip=10.0):
    """ObsNormalizer serde (normalization.rs:12-21): mean, var (Welford M2), count, clip"""
    mean, m2, count = ctx.obs_norm()
    d = {"mean": [float(x) for x in mean], "var": [float(x) for x in m2], "count": float(count), "clip": F32(clip)}
    with open(os.path.join(path_dir, "normalizer.json"), "w") as f:
        f.write(to_json_pretty(d))


def load_normalizer(ctx, path_dir):
    p = os.path.join(path_dir, "normalizer.json")
    if not os.path.exists(p):
        return False
    d = json.load(open(p))
    ctx.set_obs_norm(np.asarray(d["mean"], np.float64), np.asarray(d["var"], np.float64), float(d["count"]))
    return True


def save_return_normalizer(ctx, path_dir):
    """ReturnNormalizer serde (normalization.rs:115-135)"""
    c = ctx.cfg
    mvc, rets = ctx.ret_norm()
    P = ctx.num_players
    d = {"returns": [[float(x) for x in rets[e * P:(e + 1) * P]] for e in range(ctx.N)],
         "var": float(mvc[1]), "mean": float(mvc[0]), "count": float(mvc[2]), "gamma": float(c["gamma"]),
         "clip": F32(c["return_clip"]), "num_players": P, "epsilon": 1e-8}
    with open(os.path.join(path_dir, "return_normalizer.json"), "w") as f:
        f.write(to_json_pretty(d))


def load_return_normalizer(ctx, path_dir):
    p = os.path.join(path_dir, "return_normalizer.json")
    if not os.path.exists(p):
        return False
    d = json.load(open(p))
    rets = np.asarray(d["returns"], np.float64).reshape(-1)
    ctx.set_ret_norm(np.array([d["mean"], d["var"], d["count"]], np.float64), rets)
    return True


def save_popart_normalizer(ctx, path_dir):
    """checkpoint.rs:468-476: PopArtNormalizer serde {mean, var (M2), count, epsilon}"""
    st = ctx.popart()
    d = {"mean": float(st[0]), "var": float(st[1]), "count": float(st[2]), "epsilon": float(st[3])}
    with open(os.path.join(path_dir, "popart_normalizer.json"), "w") as f:
        f.write(to_json_pretty(d))


def load_popart_normalizer(ctx, path_dir):
    p = os.path.join(path_dir, "popart_normalizer.json")
    if not os.path.exists(p):
        return False
    d = json.load(open(p))
    ctx.set_popart([d["mean"], d["var"], d["count"], d["epsilon"]])
    return True


# -------------------------------------------------------------------- RNG ---
def save_rng_state(ctx, path_dir):
    """checkpoint.rs:390-400: 32 bytes from the main RNG (8 words) -> rng_state.bin"""
    b = (C.c_uint8 * 32)()
    ctx._chk(L.lib().bppo_rng_fill_bytes(ctx.h, b, 32))
    with open(os.path.join(path_dir, "rng_state.bin"), "wb") as f:
        f.write(bytes(b))
    return bytes(b)


def load_rng_state(ctx, path_dir):
    """checkpoint.rs:405-426: StdRng::from_seed(bytes); a wrong length is an error"""
    p = os.path.join(path_dir, "rng_state.bin")
    if not os.path.exists(p):
        return False
    seed = open(p, "rb").read()
    if len(seed) != 32:
        raise ValueError(f"Invalid RNG state file: expected 32 bytes, got {len(seed)}")
    buf = (C.c_uint8 * 32).from_buffer_copy(seed)
    ctx._chk(L.lib().bppo_rng_from_seed(ctx.h, buf))
    return True


# ---------------------------------------------------------------- manager ---
class CheckpointManager:
    """checkpoint.rs:121-272"""

    def __init__(self, run_dir):
        self.checkpoints_dir = os.path.join(run_dir, "checkpoints")
        os.makedirs(self.checkpoints_dir, exist_ok=True)
        self.best_avg_return = float("-inf")

    def save(self, ctx, params, metadata, update_best=True):
        """model + metadata with an atomic rename, then the latest / best symlinks"""
        name = f"step_{metadata.step:08d}"
        final = os.path.join(self.checkpoints_dir, name)
        tmp = os.path.join(self.checkpoints_dir, f".tmp_{name}")
        os.makedirs(tmp, exist_ok=True)
        save_model(ctx.cfg, params, os.path.join(tmp, "model.mpk"))
        with open(os.path.join(tmp, "metadata.json"), "w") as f:
            f.write(metadata.to_json())
        if os.path.exists(final):
            shutil.rmtree(final)
        os.rename(tmp, final)
        self._symlink("latest", final)
        if update_best and np.float32(metadata.avg_return) > np.float32(self.best_avg_return):
            self.best_avg_return = float(np.float32(metadata.avg_return))
            self._symlink("best", final)
        return final

    def _symlink(self, name, target):
        link = os.path.join(self.checkpoints_dir, name)
        tmp = os.path.join(self.checkpoints_dir, f".tmp_{name}")
        if os.path.lexists(tmp):
            os.remove(tmp)
        os.symlink(os.path.basename(target), tmp)
        os.rename(tmp, link)

    def set_best_checkpoint(self, name):
        d = os.path.join(self.checkpoints_dir, name)
        if not os.path.exists(d):
            raise FileNotFoundError(f"Checkpoint directory does not exist: {d}")
        self._symlink("best", d)

    @staticmethod
    def load(ckpt_dir):
        """-> (params, metadata); the architecture comes from the metadata"""
        meta = load_metadata(ckpt_dir)
        return load_model(os.path.join(ckpt_dir, "model.mpk")), meta


def save_training_checkpoint(manager, ctx, params, metadata, update_best=None):
    """one periodic checkpoint of run_training (main.rs:1276-1310): model +
    metadata, optimizer, normalizers (when on), then the RNG draw.  update_best
    defaults to use_avg_return_for_best = (num_players == 1) (main.rs:659, 1276):
    multi-player runs move 'best' through pool evaluation, not avg_return."""
    if update_best is None:
        update_best = ctx.num_players == 1
    path = manager.save(ctx, params, metadata, update_best)
    save_optimizer(ctx, path)
    if ctx.cfg["normalize_obs"]:
        save_normalizer(ctx, path)
    nr = ctx.cfg["normalize_returns"]
    if (ctx.num_players == 1) if nr is None else nr:
        save_return_normalizer(ctx, path)
    if ctx.cfg.get("normalize_values"):
        save_popart_normalizer(ctx, path)
    save_rng_state(ctx, path)
    return path


def resume_training_checkpoint(ctx, ckpt_dir):
    """the resume half (main.rs:294-414): params, optimizer, normalizers and the
    main RNG reseeded from rng_state.bin; -> metadata"""
    params, meta = CheckpointManager.load(ckpt_dir)
    ctx._chk(L.lib().bppo_params_set(ctx.h, np.ascontiguousarray(params, np.float32).ctypes.data, params.size))
    load_optimizer(ctx, ckpt_dir)
    load_normalizer(ctx, ckpt_dir)
    load_return_normalizer(ctx, ckpt_dir)
    load_popart_normalizer(ctx, ckpt_dir)
    load_rng_state(ctx, ckpt_dir)
    return meta
