"""Pin the CPU oracle (oracle/encdiff_oracle.py) to fixtures produced by the
reference implementation itself (tools/gen_golden.py)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import encdiff_oracle as O

torch.set_num_threads(min(8, os.cpu_count() or 1))


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64); b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="module")
def plan():
    return O.build_plan()


def test_param_shapes_match_reference(plan, golden_dir):
    ref = json.load(open(os.path.join(golden_dir, "unet_state_dict_shapes.json")))
    mine = {k: list(v) for k, v in O.param_shapes(plan).items()}
    assert mine == ref


def test_unet_forward_backward(plan, golden_dir):
    fx = np.load(os.path.join(golden_dir, "unet_b4.npz"))
    P = {k: v.requires_grad_(True) for k, v in O.recipe_params(O.param_shapes(plan)).items()}
    x = torch.tensor(fx["x"]).requires_grad_(True)
    ctx = torch.tensor(fx["ctx"]).requires_grad_(True)
    out = O.unet_forward(P, plan, x, torch.tensor(fx["t"]), [ctx])
    assert rel_l2(out.detach(), fx["eps"]) < 1e-5
    out.backward(torch.tensor(fx["gout"]))
    assert rel_l2(x.grad, fx["dx"]) < 1e-4
    assert rel_l2(ctx.grad, fx["dctx"]) < 1e-4
    for k in fx.files:
        if k.startswith("grad."):
            assert rel_l2(P[k[5:]].grad, fx[k]) < 1e-4, k


def test_encoder4(golden_dir):
    fx = np.load(os.path.join(golden_dir, "encoder4.npz"))
    P = O.encoder4_params()
    c = O.encoder4_forward(P, torch.tensor(fx["img"]), train=True)
    assert rel_l2(c.detach(), fx["c_train"]) < 1e-5


def test_schedule(golden_dir):
    fx = np.load(os.path.join(golden_dir, "schedule.npz"))
    d = O.register_schedule()
    for k in ["betas", "alphas_cumprod", "sqrt_alphas_cumprod", "sqrt_one_minus_alphas_cumprod",
              "posterior_variance", "posterior_mean_coef1", "posterior_mean_coef2", "lvlb_weights"]:
        np.testing.assert_array_equal(np.float32(d[k]), fx[k], err_msg=k)
    ac32 = torch.tensor(fx["alphas_cumprod"])
    for S in (10, 50, 200):
        for eta in (0, 1):
            dd = O.ddim_schedule(ac32, S, float(eta))
            np.testing.assert_array_equal(dd["timesteps"], fx[f"ddim{S}_timesteps"])
            np.testing.assert_allclose(dd["sigmas"], fx[f"ddim{S}_eta{eta}_sigmas"], rtol=1e-12, atol=0)
            np.testing.assert_allclose(dd["alphas_prev"], fx[f"ddim{S}_eta{eta}_alphas_prev"], rtol=1e-12)


def test_p_losses(plan, golden_dir):
    fx = np.load(os.path.join(golden_dir, "p_losses.npz"))
    P = O.recipe_params(O.param_shapes(plan))
    sched = O.sched_fp32(O.register_schedule())
    t = torch.tensor(fx["t"])
    noise = torch.tensor(fx["noise"])
    with torch.no_grad():
        xn = O.q_sample(sched, torch.tensor(fx["x0"]), t, noise)
        eps = O.unet_forward(P, plan, xn, t, [torch.tensor(fx["cond"])])
        loss, ld = O.p_losses_from_output(sched, eps, noise, t)
    assert rel_l2(eps, fx["eps"]) < 1e-5
    assert abs(float(loss) - float(fx["loss"])) < 1e-6
    assert abs(float(ld["loss_vlb"]) - float(fx["loss_vlb"])) < 1e-6 * max(1.0, abs(float(fx["loss_vlb"])))
    E = O.encoder4_params()
    c = O.encoder4_forward(E, torch.tensor(fx["img"]), train=True)
    assert rel_l2(c.detach(), fx["cond"]) < 1e-5


@pytest.mark.parametrize("eta", [0, 1])
def test_ddim_sampling(plan, golden_dir, eta):
    fx = np.load(os.path.join(golden_dir, "ddim.npz"))
    P = O.recipe_params(O.param_shapes(plan))
    cond = torch.tensor(fx["cond"])
    ac32 = O.sched_fp32(O.register_schedule())["alphas_cumprod"]
    torch.manual_seed(1234)
    with torch.no_grad():
        xs = O.ddim_sample(lambda x, ts: O.unet_forward(P, plan, x, ts, [cond]), torch.tensor(fx["xT"]),
                           10, float(eta), ac32)
    assert rel_l2(xs, fx[f"samples_eta{eta}"]) < 1e-4


def test_ema_adamw_lr(golden_dir):
    fx = np.load(os.path.join(golden_dir, "ema_adamw_lr.npz"))
    names = [k[5:] for k in fx.files if k.startswith("init.")]
    names.sort(key=lambda n: ["0.weight", "0.bias", "2.weight", "2.bias"].index(n))
    p = {n: torch.tensor(fx["init." + n]) for n in names}
    m = {n: torch.zeros_like(v) for n, v in p.items()}
    v2 = {n: torch.zeros_like(v) for n, v in p.items()}
    shadow = {n: t.clone() for n, t in p.items()}
    nu = 0
    gi = 0
    for step in range(1, 4):
        for n in names:
            p[n], m[n], v2[n] = O.adamw_step(p[n], torch.tensor(fx[f"grad{gi}"]), m[n], v2[n], step, 1e-3)
            gi += 1
        shadow, nu = O.ema_update(shadow, p, nu)
    for n in names:
        np.testing.assert_allclose(p[n].numpy(), fx["param." + n], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(shadow[n].numpy(), fx["ema." + n.replace(".", "")], rtol=1e-5, atol=1e-7)
    for n, f in zip(fx["lr_n"], fx["lr_f"]):
        assert abs(O.lambda_linear_schedule(int(n)) - f) < 1e-12


def test_vq_encoder_matches_reference(golden_dir):
    """Oracle VQ first-stage encode (quant_conv(Encoder(x)), autoencoder.py:313-316) vs the
    reference's own encode of the same recipe weights and images (p_losses.npz: vq_z)."""
    fx = np.load(os.path.join(golden_dir, "p_losses.npz"))
    z = O.vq_encode(O.vq_encoder_params(), torch.tensor(fx["img"]))
    assert rel_l2(z, fx["vq_z"]) < 1e-5


@pytest.mark.parametrize("eta", [0, 1])
def test_ddim_sampling_s200(plan, golden_dir, eta):
    """The reference's log_images length (ddpm_enc.py:1474: ddim_steps=200, ddim_eta=1.): oracle
    samples and the logged intermediates vs the reference's own (ddim_s200.npz)."""
    fx = np.load(os.path.join(golden_dir, "ddim_s200.npz"))
    P = O.recipe_params(O.param_shapes(plan))
    cond = torch.tensor(fx["cond"])
    ac32 = O.sched_fp32(O.register_schedule())["alphas_cumprod"]
    torch.manual_seed(1234)
    with torch.no_grad():
        xs, inter = O.ddim_sample(lambda x, ts: O.unet_forward(P, plan, x, ts, [cond]), torch.tensor(fx["xT"]),
                                  200, float(eta), ac32, log_every_t=100)
    assert rel_l2(xs, fx[f"samples_eta{eta}"]) < 1e-4
    assert len(inter["x_inter"]) == fx[f"x_inter_eta{eta}"].shape[0]
    assert rel_l2(torch.stack(inter["x_inter"]), fx[f"x_inter_eta{eta}"]) < 1e-4
    assert rel_l2(torch.stack(inter["pred_x0"]), fx[f"pred_x0_eta{eta}"]) < 1e-4
