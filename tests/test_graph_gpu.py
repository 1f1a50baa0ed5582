"""HIP-graph capture of a whole data-parallel training step.

One MI355X, one process as rank 0 of an emulated 8-rank DP job (loopback DP group,
comm/loopback.py: the reduce-scatter / all-gather stand-ins run on the group's side stream as an
RCCL collective would). The step — forward, backward with the framework DDP's bucketed gradient
reductions, the hand-written fused Adam with its device-side step count (optim.hip
``adam_capturable``), and for ZeRO-1 the parameter all-gather — is captured once and replayed;
parameters after the replays equal the same steps run eagerly.
"""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _model():
    torch.manual_seed(3)
    return nn.Sequential(nn.Conv2d(3, 16, 3, padding=1), nn.ReLU(), nn.AdaptiveAvgPool2d(4), nn.Flatten(),
                         nn.Linear(256, 64), nn.ReLU(), nn.Linear(64, 10)).cuda()


def _run(zero, graph, steps=4):
    from smdt_amd.optim.optimizer import MixedPrecisionAdam
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel as DDP
    ps.destroy_model_parallel()
    ps.initialize_emulated_tensor_parallel(1, 8)
    ddp = DDP(_model(), torch_compat=True, bucket_size=4096, use_distributed_optimizer=zero)
    assert ddp.dp == 8
    opt = MixedPrecisionAdam(ddp, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, adamw=False,
                             capturable=True)
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(16, 3, 8, 8, device="cuda", generator=g)
    y = torch.randint(0, 10, (16,), device="cuda", generator=g)
    crit = nn.CrossEntropyLoss()

    def step():
        loss = crit(ddp(x), y)
        loss.backward()
        opt.step()
        ddp.wait_param_gather()            # ZeRO-1: the all-gather completes inside the step
        return loss

    if not graph:
        losses = [step().item() for _ in range(steps)]
    else:
        step()                             # one eager step (algorithm selection, buffers)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            static_loss = step()
        losses = [None]                    # (the capture itself ran no kernels)
        for _ in range(steps - 1):
            gr.replay()
            losses.append(static_loss.item())
    torch.cuda.synchronize()
    params = [p.detach().clone() for p in ddp.module.parameters()]
    st = opt.state_dict()["step"]
    ps.destroy_model_parallel()
    return losses, params, st


@pytest.mark.parametrize("zero", [False, True])
def test_captured_emulated_dp8_step_equals_eager(zero):
    le, pe, se = _run(zero, graph=False)
    lg, pg, sg = _run(zero, graph=True)
    assert se == sg == 4                   # the device step count advanced on every replay
    for a, b in zip(le[1:], lg[1:]):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (le, lg)
    for a, b in zip(pe, pg):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
