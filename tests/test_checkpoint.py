"""Checkpoint interop (checkpoint.rs) host side, CPU: serde_json pretty layout
with ryu floats, CheckpointMetadata required fields / serde defaults
(checkpoint.rs:26-96), the model / optimizer MessagePack records round trip,
and CheckpointManager's atomic save + latest / best symlinks
(checkpoint.rs:147-189, tests 502-700)."""
import json
import os

import numpy as np
import pytest

import bppo
from bppo import checkpoint as K


@pytest.mark.parametrize("v,f32,text", [
    (1.0, False, "1.0"), (0.1, False, "0.1"), (1e-8, False, "1e-8"), (1e-5, False, "0.00001"),
    (1e-6, False, "1e-6"), (123456789.0, False, "123456789.0"), (1e16, False, "1e16"), (1e15, False, "1000000000000000.0"),
    (1e17, False, "1e17"), (1.5e-7, False, "1.5e-7"), (-2.5, False, "-2.5"), (0.99, False, "0.99"),
    (0.99, True, "0.99"), (475.0, True, "475.0"), (0.1, True, "0.1"), (1.2345678e20, False, "1.2345678e20"),
    (float("nan"), False, "null"), (float("-inf"), True, "null"), (0.0, False, "0.0")])
def test_ryu_float_text(v, f32, text):
    assert K.to_json_pretty(K.F32(v) if f32 else v) == text


def test_pretty_layout():
    assert K.to_json_pretty({"a": [1, 2], "b": {}, "c": [], "d": None, "e": "x"}) == \
        '{\n  "a": [\n    1,\n    2\n  ],\n  "b": {},\n  "c": [],\n  "d": null,\n  "e": "x"\n}'


def _meta(step=1000, ret=150.0):
    return K.CheckpointMetadata(step=step, avg_return=ret, rng_seed=42, best_avg_return=ret,
                                recent_returns=[140.0, 150.0, 160.0], obs_dim=4, action_count=2, num_players=1,
                                hidden_size=64, num_hidden=2, activation="tanh", env_name="cartpole")


def test_metadata_round_trip_and_field_order():
    m = _meta()
    text = m.to_json()
    d = json.loads(text)
    assert list(d)[:6] == ["step", "avg_return", "rng_seed", "best_avg_return", "recent_returns", "forked_from"]
    assert list(d)[-2:] == ["env_name", "exploitability_vs_pool"]
    assert K.CheckpointMetadata.from_json(text) == m


def test_metadata_required_fields_and_defaults():
    d = json.loads(_meta().to_json())
    for k in ("split_networks", "network_type", "conv_channels", "obs_shape"):   # #[serde(default)]
        d.pop(k)
    m = K.CheckpointMetadata.from_json(json.dumps(d))
    assert m.network_type == "mlp" and m.conv_channels == [64, 64] and m.obs_shape is None
    d.pop("obs_dim")                                                           # required
    with pytest.raises(ValueError):
        K.CheckpointMetadata.from_json(json.dumps(d))
    d = json.loads(_meta().to_json())
    d["global_state_dim"] = d.pop("privileged_obs_dim")                      # serde alias
    assert K.CheckpointMetadata.from_json(json.dumps(d)).privileged_obs_dim is None


@pytest.mark.parametrize("preset,over", [("cartpole", {}), ("connect_four", {}), ("liars_dice_ctde", {}),
                                         ("connect_four", {"network_type": "cnn"}),
                                         ("cartpole", {"split_networks": True, "hidden_size": 32, "num_hidden": 3}),
                                         ("liars_dice_ctde", {"network_type": "mlp", "hidden_size": 128}),
                                         ("connect_four", {"network_type": "cnn", "split_networks": True})])
def test_model_record_round_trip(tmp_path, preset, over):
    cfg = bppo.make_config(preset, **over)
    p = bppo.orthogonal_init(cfg, seed=3)
    path = str(tmp_path / "model.mpk")
    K.save_model(cfg, p, path)
    q = K.load_model(path)
    assert q.dtype == np.float32 and np.array_equal(p.view(np.uint32), q.view(np.uint32))
    rec = K.model_record(cfg, p)
    assert set(rec) == {"metadata", "item"} and rec["metadata"]["float"] == "f32"
    (kind, body), = rec["item"].items()
    assert kind == {"ctde": "Ctde", "cnn": "Cnn", "mlp": "Mlp"}[cfg["network_type"]]
    lin = body["policy_head"]
    assert set(lin) == {"weight", "bias"} and lin["weight"]["param"]["dtype"] == "F32"
    if cfg.get("split_networks") and kind == "Mlp":   # mlp.rs:47-62: critic_layers on obs, same widths
        assert [c["weight"]["param"]["shape"] for c in body["critic_layers"]] == \
            [[5, 32], [32, 32], [32, 32]]
    if kind == "Cnn":   # cnn.rs:24-50: critic stacks only with split_networks, same shapes as the actor's
        shapes = lambda layers: [c["weight"]["param"]["shape"] for c in layers]
        assert shapes(body["conv_layers"]) == [[8, 2, 3, 3], [8, 8, 3, 3]]
        split = bool(cfg.get("split_networks"))
        assert shapes(body["critic_conv_layers"]) == (shapes(body["conv_layers"]) if split else [])
        assert shapes(body["critic_fc_layers"]) == (shapes(body["fc_layers"]) if split else [])


def test_optimizer_record_round_trip():
    cfg = bppo.make_config("cartpole")
    n = bppo.orthogonal_init(cfg).size
    rng = np.random.default_rng(0)
    m1, m2 = rng.normal(size=n).astype(np.float32), rng.random(n).astype(np.float32)
    steps = np.arange(8, dtype=np.int32) + 3
    rec, ids = K.optimizer_record(cfg, m1, m2, steps)
    assert len(ids) == 8 and len(set(ids)) == 8
    got = np.concatenate([np.frombuffer(rec["item"][i]["momentum"]["moment_1"]["bytes"], np.float32) for i in ids])
    assert np.array_equal(got, m1)
    assert [rec["item"][i]["momentum"]["time"] for i in ids] == list(steps)


@pytest.mark.parametrize("preset,over", [("cartpole", {}), ("liars_dice_ctde", {}),
                                         ("connect_four", {"network_type": "cnn"}),
                                         ("connect_four", {"network_type": "cnn", "split_networks": True})])
def test_optimizer_moment_shapes_match_model_record(preset, over):
    """each Adam moment has the shape of its parameter in the model record
    (Conv2d weights [Cout, Cin, k, k], critic conv stacks included), as Burn's state
    mirrors the gradient; the flat moments round-trip through the record."""
    cfg = bppo.make_config(preset, **over)
    p = bppo.orthogonal_init(cfg, seed=1)
    rng = np.random.default_rng(1)
    m1, m2 = rng.normal(size=p.size).astype(np.float32), rng.random(p.size).astype(np.float32)
    steps = np.arange(2 * len(bppo.host.layer_shapes(cfg)[0]), dtype=np.int32)
    rec, ids = K.optimizer_record(cfg, m1, m2, steps)
    model = K.model_record(cfg, p)["item"]
    params = [lin[k] for lin in K._linears_in_order(model) for k in ("weight", "bias")]
    assert ids == [q["id"] for q in params]
    for q in params:
        st = rec["item"][q["id"]]["momentum"]
        assert st["moment_1"]["shape"] == q["param"]["shape"] == st["moment_2"]["shape"]
    a1, a2, st = K.optimizer_arrays(rec, ids)
    assert np.array_equal(a1, m1) and np.array_equal(a2, m2) and np.array_equal(st, steps)


def test_optimizer_read_with_the_model_record_ids(tmp_path):
    """Burn keys optimizer.mpk by the model's random ParamIds: a record written
    with ids unknown to this module loads through the ids of model.mpk beside it."""
    import msgpack
    cfg = bppo.make_config("cartpole")
    p = bppo.orthogonal_init(cfg)
    rec = K.model_record(cfg, p)
    rng = np.random.default_rng(9)
    fresh = [str(int(x)) for x in rng.integers(1, 2**48, 8)]
    lins = K._linears_in_order(rec["item"])
    for t, (lin, k) in enumerate((lin, k) for lin in lins for k in ("weight", "bias")):
        lin[k]["id"] = fresh[t]
    (tmp_path / "model.mpk").write_bytes(msgpack.packb(rec, use_bin_type=True))
    assert K.model_param_ids(str(tmp_path)) == fresh
    n = p.size
    m1, m2 = rng.normal(size=n).astype(np.float32), rng.random(n).astype(np.float32)
    steps = np.arange(8, dtype=np.int32) + 5
    orec, hashed = K.optimizer_record(cfg, m1, m2, steps)
    orec["item"] = {fresh[i]: orec["item"][h] for i, h in enumerate(hashed)}    # as the reference writes it
    a1, a2, st = K.optimizer_arrays(orec, K.model_param_ids(str(tmp_path)))
    assert np.array_equal(a1, m1) and np.array_equal(a2, m2) and list(st) == list(steps)
    with pytest.raises(KeyError):
        K.optimizer_arrays(orec, hashed)
    assert K.model_param_ids(str(tmp_path / "missing")) is None


def _ref_meta(obs_dim, action_count, num_players, env_name, **kw):
    """what main.rs:451-476 writes: every config field as given (config.rs defaults
    num_conv_layers 2, conv_channels [8, 8], kernel_size 3, cnn_fc_hidden_size 32,
    cnn_num_fc_layers 1), obs_shape = E::OBSERVATION_SHAPE"""
    d = dict(step=0, avg_return=0.0, rng_seed=42, best_avg_return=None, recent_returns=[], forked_from=None,
             obs_dim=obs_dim, action_count=action_count, num_players=num_players, hidden_size=64, num_hidden=2,
             activation="relu", split_networks=False, network_type="mlp", num_conv_layers=2, conv_channels=[8, 8],
             kernel_size=3, cnn_fc_hidden_size=32, cnn_num_fc_layers=1, privileged_obs_dim=None,
             critic_hidden_size=None, critic_num_hidden=None, obs_shape=None, env_name=env_name,
             exploitability_vs_pool=None)
    d.update(kw)
    return d


@pytest.mark.parametrize("preset,over,ref", [
    ("cartpole", {}, _ref_meta(5, 2, 1, "cartpole")),
    ("connect_four", {}, _ref_meta(86, 7, 2, "connect_four", hidden_size=512, obs_shape=[6, 7, 2])),
    ("connect_four", {"network_type": "cnn", "conv_channels": [64]},
     _ref_meta(86, 7, 2, "connect_four", hidden_size=512, network_type="cnn", conv_channels=[64], obs_shape=[6, 7, 2])),
    ("liars_dice_ctde", {}, _ref_meta(270, 49, 4, "liars_dice", hidden_size=256, network_type="ctde",
                                      privileged_obs_dim=120, critic_hidden_size=512, critic_num_hidden=3)),
    ("liars_dice_ctde", {"network_type": "mlp", "split_networks": True},
     _ref_meta(270, 49, 4, "liars_dice", hidden_size=256, split_networks=True, critic_hidden_size=512,
               critic_num_hidden=3)),
])
def test_for_config_writes_the_reference_metadata(preset, over, ref):
    """CheckpointMetadata::for_config vs the fields main.rs:451-476 writes"""
    cfg = bppo.make_config(preset, **over)
    got = json.loads(K.CheckpointMetadata.for_config(cfg, 0, 0.0).to_json())
    assert got == ref


class _FakeCtx:
    def __init__(self, cfg):
        self.cfg = cfg


def test_manager_best_and_latest_symlinks(tmp_path):          # checkpoint.rs:565-640
    cfg = bppo.make_config("cartpole")
    mgr = K.CheckpointManager(str(tmp_path))
    p = bppo.orthogonal_init(cfg)
    ctx = _FakeCtx(cfg)
    for step, ret in ((1000, 100.0), (2000, 200.0), (3000, 150.0)):
        mgr.save(ctx, p, _meta(step, ret))
    ck = tmp_path / "checkpoints"
    assert os.readlink(ck / "latest") == "step_00003000"
    assert os.readlink(ck / "best") == "step_00002000"
    params, meta = K.CheckpointManager.load(str(ck / "best"))
    assert meta.step == 2000 and meta.avg_return == 200.0 and np.array_equal(params, p)
    assert not any(x.name.startswith(".tmp_") for x in ck.iterdir())
    mgr.set_best_checkpoint("step_00001000")
    assert os.readlink(ck / "best") == "step_00001000"
    with pytest.raises(FileNotFoundError):
        mgr.set_best_checkpoint("step_00009999")
