"""The oracle's hand-written PPO loss backward (oracle/net.c, restating
ppo.rs:1385-1502 + Burn autodiff) checked against torch CPU autograd of the
same loss expression in float64."""
import ctypes as C

import numpy as np
import pytest
import torch

import oracle_ffi as O


def layer_shapes(desc):
    shapes = []
    i = desc.obs_dim
    if desc.cnn:
        cin = desc.C
        for l in range(desc.n_conv):
            shapes.append((cin * desc.ksize ** 2, desc.conv_ch[l])); cin = desc.conv_ch[l]
        i = desc.H * desc.W * cin + desc.obs_dim - desc.H * desc.W * desc.C
    for _ in range(desc.n_actor):
        shapes.append((i, desc.actor_width)); i = desc.actor_width
    if desc.split and desc.cnn:   # cnn.rs:24-50 record: conv, fc, critic conv, critic fc, heads
        return shapes + shapes + [(i, desc.act_dim), (i, 1)]
    if desc.split:   # mlp.rs:47-62 record: layers, critic_layers, policy_head, value_head
        c = desc.obs_dim
        for _ in range(desc.n_critic):
            shapes.append((c, desc.critic_width)); c = desc.critic_width
        return shapes + [(i, desc.act_dim), (c, 1)]
    shapes.append((i, desc.act_dim))
    if desc.ctde:
        c = desc.priv_dim + desc.obs_dim
        for _ in range(desc.n_critic):
            shapes.append((c, desc.critic_width)); c = desc.critic_width
        shapes.append((c, 1))
    else:
        shapes.append((i, 1))
    return shapes


def torch_loss(desc, params, obs, priv, actions, old_logp, adv_n, returns, old_values, masks,
               clip=0.2, vcoef=0.5, ent=0.01, clip_value=False):
    p = torch.tensor(params, dtype=torch.float64, requires_grad=True)
    off = 0
    Ws = []
    for (i, o) in layer_shapes(desc):
        W = p[off:off + i * o].view(i, o); off += i * o
        b = p[off:off + o]; off += o
        Ws.append((W, b))
    act = torch.relu if desc.relu else torch.tanh
    x = torch.tensor(obs, dtype=torch.float64)
    h = x

    def conv_stack(convs):
        # cnn.rs:241-330: obs[:, :HWC] reshaped [B, H, W, C] and permuted to NCHW,
        # conv (weight [Cout][Cin][k][k], same padding) + relu, flatten NCHW, cat extra
        Hh, Ww, Cc = desc.H, desc.W, desc.C
        sp = x[:, :Hh * Ww * Cc].reshape(-1, Hh, Ww, Cc).permute(0, 3, 1, 2)
        cin = Cc
        for l, (W, b) in enumerate(convs):
            co = desc.conv_ch[l]
            sp = torch.relu(torch.nn.functional.conv2d(sp, W.reshape(co, cin, desc.ksize, desc.ksize), b,
                                                       padding=desc.ksize // 2))
            cin = co
        return torch.cat([sp.reshape(sp.shape[0], -1), x[:, Hh * Ww * Cc:]], 1)
    if desc.cnn and desc.split:   # cnn.rs:264-302: two conv+FC trunks on the same input
        nt = desc.n_conv + desc.n_actor
        h, hc = conv_stack(Ws[:desc.n_conv]), conv_stack(Ws[nt:nt + desc.n_conv])
        for W, b in Ws[desc.n_conv:nt]:
            h = act(h @ W + b)
        for W, b in Ws[nt + desc.n_conv:2 * nt]:
            hc = act(hc @ W + b)
        logits = h @ Ws[2 * nt][0] + Ws[2 * nt][1]
        v = (hc @ Ws[-1][0] + Ws[-1][1])[:, 0]
        return _loss_tail(logits, v, actions, old_logp, adv_n, returns, old_values, masks, clip, vcoef, ent,
                          clip_value, p)
    if desc.cnn:
        h = conv_stack(Ws[:desc.n_conv])
        Ws = Ws[desc.n_conv:]
    if desc.split:   # mlp.rs:143-185: actor trunk -> policy, critic trunk on obs -> value
        na, nc = desc.n_actor, desc.n_critic
        for W, b in Ws[:na]:
            h = act(h @ W + b)
        hc = x
        for W, b in Ws[na:na + nc]:
            hc = act(hc @ W + b)
        logits = h @ Ws[na + nc][0] + Ws[na + nc][1]
        v = (hc @ Ws[-1][0] + Ws[-1][1])[:, 0]
        return _loss_tail(logits, v, actions, old_logp, adv_n, returns, old_values, masks, clip, vcoef, ent,
                          clip_value, p)
    for W, b in Ws[:desc.n_actor]:
        h = act(h @ W + b)
    logits = h @ Ws[desc.n_actor][0] + Ws[desc.n_actor][1]
    if desc.ctde:
        hc = torch.cat([torch.tensor(priv, dtype=torch.float64), x], 1)
        for W, b in Ws[desc.n_actor + 1:-1]:
            hc = act(hc @ W + b)
        v = (hc @ Ws[-1][0] + Ws[-1][1])[:, 0]
    else:
        v = (h @ Ws[-1][0] + Ws[-1][1])[:, 0]
    return _loss_tail(logits, v, actions, old_logp, adv_n, returns, old_values, masks, clip, vcoef, ent,
                      clip_value, p)


def _loss_tail(logits, v, actions, old_logp, adv_n, returns, old_values, masks, clip, vcoef, ent, clip_value, p):
    if masks is not None:
        logits = logits + (torch.tensor(masks, dtype=torch.float64) - 1.0) * 1e9
    ls = torch.log_softmax(logits, 1)
    newlp = ls.gather(1, torch.tensor(actions, dtype=torch.long)[:, None])[:, 0]
    H = -(ls.exp() * ls).sum(1)
    ratio = torch.exp(newlp - torch.tensor(old_logp, dtype=torch.float64))
    na = -torch.tensor(adv_n, dtype=torch.float64)
    pl = torch.maximum(na * ratio, na * ratio.clamp(1 - clip, 1 + clip)).mean()
    R = torch.tensor(returns, dtype=torch.float64)
    if clip_value:
        vo = torch.tensor(old_values, dtype=torch.float64)
        vc = vo + (v - vo).clamp(-clip, clip)
        vl = torch.maximum((v - R) ** 2, (vc - R) ** 2).mean() * 0.5
    else:
        vl = ((v - R) ** 2).mean() * 0.5
    loss = pl + vl * vcoef - H.mean() * ent
    loss.backward()
    return loss.item(), p.grad.numpy()


def run_case(desc, mb, masks=False, seed=0, clip_value=False):
    rng = np.random.default_rng(seed)
    params = (rng.normal(size=desc.n_params) * 0.3).astype(np.float32)
    obs = rng.normal(size=(mb, desc.obs_dim)).astype(np.float32)
    priv = rng.normal(size=(mb, desc.priv_dim)).astype(np.float32) if desc.ctde else None
    A = desc.act_dim
    mk = None
    if masks:
        mk = (rng.random((mb, A)) < 0.6).astype(np.float32)
        mk[np.arange(mb), rng.integers(0, A, mb)] = 1.0
    actions = np.array([rng.choice(np.flatnonzero(mk[i])) if masks else rng.integers(0, A)
                        for i in range(mb)], np.int32)
    old_logp = (rng.normal(size=mb) * 0.3 - 1.0).astype(np.float32)
    adv = rng.normal(size=mb).astype(np.float32)
    ret = rng.normal(size=mb).astype(np.float32)
    ov = rng.normal(size=mb).astype(np.float32)
    cfg = O.ppo_cfg(clip_value=clip_value)
    grads = np.zeros(desc.n_params, np.float32)
    st = O.MbStats()
    O.lib().or_minibatch_loss_grad(C.byref(desc), params, mb, obs,
                                   None if priv is None else priv.ctypes.data, actions, old_logp,
                                   adv, ret, ov, None if mk is None else mk.ctypes.data,
                                   C.byref(cfg), 0.01, grads, C.byref(st))
    loss_t, g_t = torch_loss(desc, params, obs, priv, actions, old_logp, adv, ret, ov, mk,
                             clip_value=clip_value)
    assert abs(st.loss - loss_t) <= 1e-5 * max(1.0, abs(loss_t))
    scale = np.abs(g_t).max()
    np.testing.assert_allclose(grads, g_t, rtol=0, atol=2e-5 * scale)


def test_mlp_cartpole_shape():
    run_case(O.mlp_desc(5, 2, 64, 2), mb=257)


def test_mlp_masked_connect_four_shape():
    run_case(O.mlp_desc(86, 7, 32, 2), mb=129, masks=True, seed=1)


def test_ctde_liars_dice_shape():
    run_case(O.ctde_desc(270, 120, 49, 32, 2, 48, 3), mb=65, masks=True, seed=2)


def test_clip_value_branch():
    run_case(O.mlp_desc(5, 2, 16, 1), mb=200, seed=3, clip_value=True)


def test_tanh_activation():
    run_case(O.mlp_desc(5, 2, 16, 2, relu=False), mb=100, seed=4)


def test_cnn_connect_four_shape():
    """network/cnn.rs: 2 conv layers (8, 16 channels), 3x3 same, 1 FC layer of 24"""
    run_case(O.cnn_desc(7, [8, 16], 3, 24, 1), mb=33, masks=True, seed=5)


def test_split_networks_cartpole_shape():
    """mlp.rs split_networks: actor and critic trunks of 2 x 32 on obs"""
    run_case(O.mlp_desc(5, 2, 32, 2, split=True), mb=150, seed=7)


def test_split_networks_masked_tanh():
    run_case(O.mlp_desc(86, 7, 24, 3, relu=False, split=True), mb=70, masks=True, seed=8)


def test_cnn_split_networks_shape():
    """cnn.rs:116-135 split_networks: the critic's own conv stack and FC layers"""
    run_case(O.cnn_desc(7, [8, 16], 3, 24, 1, split=True), mb=29, masks=True, seed=8)


def test_cnn_one_conv_tanh_fc_kernel5():
    run_case(O.cnn_desc(7, [6], 5, 16, 2, relu=False), mb=20, masks=True, seed=6)
