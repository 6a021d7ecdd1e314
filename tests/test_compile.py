"""torch.compile surface of the drop-in MainModel (SURVEY.md §8(b) "harness
behaviours to survive"): ``model_test.py:64`` compiles the model,
``training_tools.py:39`` with ``dynamic=True``, ``cifar100_test.py:93`` with
``fullgraph=True``.  Under compilation the fused forward is one custom op
(``sdpnet::main_forward``, sdpnet_ops.py) with a shape-only fake.

CPU tests trace with fake CUDA tensors (FakeTensorMode; no GPU or kernel runs):
one graph, zero graph breaks, correct output shapes/dtypes.  The GPU test
compiles for real and compares with the eager fused forward.
"""
import copy

import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import model as ours
import sdpnet_ops

XXS = dict(embedding_dim=64, num_blocks=2, n_head=4, patch_size=16, conv_kernel_size=7,
           head_output_from_register=True, output_classes=10)


def _model(**kw):
    cfg = dict(XXS)
    cfg.update(kw)
    return ours.MainModel(**cfg).eval()


def _export(m, x, **kw):
    gm, _ = torch._dynamo.export(m, **kw)(x)
    return gm


def _sdp_nodes(gm):
    return [n for n in gm.graph.nodes if n.op == "call_function" and "sdpnet" in str(n.target)]


def test_fullgraph_single_custom_op():
    m = _model()
    with FakeTensorMode(allow_non_fake_inputs=True):
        x = torch.empty(2, 3, 224, 224, device="cuda")
        gm = _export(m, x)
    nodes = _sdp_nodes(gm)
    assert len(nodes) == 1 and nodes[0].target in (torch.ops.sdpnet.main_forward, torch.ops.sdpnet.main_forward.default)
    calls = [n for n in gm.graph.nodes if n.op == "call_function"]
    assert calls == nodes  # nothing else traced: the whole forward is the op


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_compiled_fake_shapes(dt):
    torch._dynamo.reset()
    m = _model()
    graphs = []

    def backend(gm, example_inputs):
        graphs.append(gm)
        return gm.forward

    cm = torch.compile(m, fullgraph=True, dynamic=True, backend=backend)
    with FakeTensorMode(allow_non_fake_inputs=True):
        for B in (2, 5):
            x = torch.empty(B, 3, 224, 224, device="cuda", dtype=dt)
            y = cm(x)
            assert tuple(y.shape) == (B, 10) and y.dtype == dt and y.is_cuda
            logits, xo, regs = cm(x, return_raw_outputs=True)
            assert tuple(logits.shape) == (B, 10)
            assert tuple(xo.shape) == (B, 64, 14, 14) and xo.dtype == dt
            assert tuple(regs.shape) == (B, 4, 64)  # num_registers=3 -> 4 rows (layers.py:157)
            _, _, regs1 = cm(x, num_registers=1, return_raw_outputs=True)
            assert tuple(regs1.shape) == (B, 2, 64)
    # dynamic=True: one graph per (return_raw_outputs, num_registers) variant, reused across B
    assert 1 <= len(graphs) <= 3
    for gm in graphs:
        assert len(_sdp_nodes(gm)) == 1


@pytest.mark.gpu  # torch.autocast("cuda") disables itself without a device
def test_autocast_selects_bf16_op():
    m = _model()
    with FakeTensorMode(allow_non_fake_inputs=True):
        x = torch.empty(2, 3, 224, 224, device="cuda")
        with torch.autocast("cuda", dtype=torch.bfloat16):
            gm = _export(m, x)
    (node,) = _sdp_nodes(gm)
    assert node.args[3] == sdpnet_ops.DTYPE_CODES[torch.bfloat16]


def test_handles_follow_copies():
    m = _model()
    m2 = copy.deepcopy(m)
    assert m2._sdp_handle != m._sdp_handle
    assert sdpnet_ops.lookup(m._sdp_handle) is m
    assert sdpnet_ops.lookup(m2._sdp_handle) is m2
    h = m2._sdp_handle
    del m2
    import gc
    gc.collect()
    with pytest.raises(RuntimeError, match="not live"):
        sdpnet_ops.lookup(h)


def test_op_has_no_cpu_kernel():
    m = _model()
    x = torch.zeros(1, 3, 224, 224)
    with pytest.raises(NotImplementedError):
        torch.ops.sdpnet.main_forward(x, m._sdp_handle, 3, 0)


@pytest.mark.gpu
def test_compiled_equals_eager_on_gpu():
    torch.manual_seed(0)
    m = _model().to("cuda")
    x = torch.randn(3, 3, 224, 224, device="cuda")
    ref = m(x)
    torch._dynamo.reset()
    cm = torch.compile(m, fullgraph=True)
    y = cm(x)
    torch.testing.assert_close(y, ref, rtol=0, atol=0)
    ref_raw = m(x.bfloat16(), return_raw_outputs=True)
    y_raw = cm(x.bfloat16(), return_raw_outputs=True)
    for a, b in zip(y_raw, ref_raw):
        torch.testing.assert_close(a, b, rtol=0, atol=0)


# --------------------------------------------------------------- training mode under compile
def test_train_mode_fullgraph_single_op_pair(monkeypatch):
    """model.train() under torch.compile with SDPNET_COMPILE_TRAIN_OPS=model: the forward is one
    sdpnet::train_forward op taking the parameters, so Dynamo sees no graph break; its autograd
    formula is the sdpnet::train_backward op."""
    monkeypatch.setattr(ours, "_COMPILE_TRAIN_OPS", "model")
    m = _model(ffn_dropout=0.2, attn_dropout=0.2).train()
    with FakeTensorMode(allow_non_fake_inputs=True):
        x = torch.empty(2, 3, 224, 224, device="cuda")
        gm = _export(m, x)
    nodes = _sdp_nodes(gm)
    assert len(nodes) == 2 or len(nodes) == 1  # the op (+ its getitem when exported)
    assert any("train_forward" in str(n.target) for n in nodes)
    assert "train_backward" in str(torch.ops.sdpnet.train_backward)


@pytest.mark.parametrize("conv_first", [True, False])
def test_train_mode_fullgraph_one_op_per_sublayer(conv_first):
    """model.train() under torch.compile (training_tools.py:36-39 compiles DDP(model),
    dynamic=True; cifar100_test.py:93 fullgraph=True), the default: one sdpnet::train_layer op
    per patch-embedding / ConvMixer / EncoderLayer / head in execution order, nothing else
    traced, 0 graph breaks; every parameter of the model is an input of exactly one op."""
    import sdpnet_train
    m = _model(ffn_dropout=0.2, attn_dropout=0.2, conv_first=conv_first).train()
    with FakeTensorMode(allow_non_fake_inputs=True):
        x = torch.empty(2, 3, 224, 224, device="cuda")
        gm = _export(m, x)
    layers = sdpnet_train.train_layers(m)
    ops = [n for n in _sdp_nodes(gm) if "train_layer" in str(n.target)]
    assert len(ops) == len(layers) == 1 + len(m.blocks) * (len(m.blocks[0].conv_blocks) + 1) + 2
    assert [n.args[3] for n in ops] == list(range(len(layers)))   # layer index, in order
    kinds = [k for k, _ in layers]
    assert kinds[0] == "embed" and kinds[-1] == "head" and kinds[-2] == "enc"
    assert kinds[1] == ("mixer" if conv_first else "enc")
    seen = [id(p) for n in ops for p in n.args[1]]
    assert len(seen) == len(set(seen))  # no parameter in two layers
    assert "train_layer_backward" in str(torch.ops.sdpnet.train_layer_backward)


def test_train_mode_raw_outputs_and_image_grad_trace_fullgraph():
    """model.train() under torch.compile with return_raw_outputs=True and an image that requires grad
    (both refused before round 6): one train_layer op per sub-layer, the head as train_head_raw (logits,
    x_raw_output, registers), layer 0 told that its image needs a gradient, 0 graph breaks."""
    m = _model(ffn_dropout=0.2).train()
    with FakeTensorMode(allow_non_fake_inputs=True):
        x = torch.empty(2, 3, 224, 224, device="cuda", requires_grad=True)
        gm, _ = torch._dynamo.export(lambda t: m(t, return_raw_outputs=True))(x)
    nodes = _sdp_nodes(gm)
    layers = [n for n in nodes if "train_layer" in str(n.target)]
    heads = [n for n in nodes if "train_head_raw" in str(n.target)]
    assert len(heads) == 1 and len(layers) == len(__import__("sdpnet_train").train_layers(m)) - 1
    assert layers[0].args[7] == 1 and all(n.args[7] == 0 for n in layers[1:])  # need_dx on layer 0 only
    assert len(heads[0].args) == 9  # ..., batch, hp, wp: the image grid of the raw output (symbolic here)
    # the graph returns the head op's first three outputs: logits [B, 10], x_raw [B, C, hp, wp], registers [B, R, C]
    out = [n for n in gm.graph.nodes if n.op == "output"][0]
    assert len(out.args[0]) == 3


@pytest.mark.gpu
@pytest.mark.parametrize("bf16", [False, True])
def test_compiled_train_raw_outputs_and_image_grad_equal_eager(bf16):
    """Compiled training (fullgraph=True, dynamic=True) with return_raw_outputs=True and an image
    that requires grad: logits, raw outputs, every parameter gradient and the image gradient equal
    the eager training path's bit for bit (reference model.py:145-149 returns the raw outputs)."""
    import torch.nn.functional as F
    torch.manual_seed(0)
    m = _model(ffn_dropout=0.2, attn_dropout=0.2, stochastic_depth_p=[0.1, 0.2]).to("cuda").train()
    x0 = torch.randn(3, 3, 224, 224, device="cuda")
    y = torch.randint(0, 10, (3,), device="cuda")

    def step(mod):
        m.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        torch.manual_seed(7)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
            logits, xo, regs = mod(x, return_raw_outputs=True)
        loss = F.cross_entropy(logits.float(), y) + 0.1 * xo.float().square().mean() + regs.float().mean()
        loss.backward()
        grads = {k: (p.grad.clone() if p.grad is not None else torch.zeros_like(p)) for k, p in m.named_parameters()}
        return loss.detach(), logits.detach(), xo.detach(), regs.detach(), x.grad.clone(), grads

    eager = step(m)
    torch._dynamo.reset()
    comp = step(torch.compile(m, fullgraph=True, dynamic=True))
    for a, b, what in zip(eager[:5], comp[:5], ("loss", "logits", "x_raw", "registers", "image grad")):
        assert a.shape == b.shape and torch.equal(a, b), what
    assert eager[4].abs().sum() > 0
    for k in eager[5]:
        assert torch.equal(eager[5][k], comp[5][k]), k
    import sdpnet_ops
    assert not sdpnet_ops._TAPES


@pytest.mark.gpu
@pytest.mark.parametrize("ops", ["layer", "model"])
@pytest.mark.parametrize("bf16", [False, True])
def test_compiled_train_step_equals_eager_on_gpu(bf16, ops, monkeypatch):
    """A compiled training step (fullgraph=True, dynamic=True; loss outside the model as in
    cifar100_test.py:136-140) gives the eager step's loss and every gradient bit for bit,
    dropout and drop path active (same seeds -> same masks)."""
    import torch.nn.functional as F
    monkeypatch.setattr(ours, "_COMPILE_TRAIN_OPS", ops)
    torch.manual_seed(0)
    m = _model(ffn_dropout=0.2, attn_dropout=0.2, stochastic_depth_p=[0.1, 0.2]).to("cuda").train()
    x = torch.randn(4, 3, 224, 224, device="cuda")
    y = torch.randint(0, 10, (4,), device="cuda")

    def step(mod):
        m.zero_grad(set_to_none=True)
        torch.manual_seed(7)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
            out = mod(x)
        loss = F.cross_entropy(out.float(), y, label_smoothing=0.1)
        loss.backward()
        return loss.detach(), {k: (p.grad.clone() if p.grad is not None else torch.zeros_like(p))
                               for k, p in m.named_parameters()}

    l_eager, g_eager = step(m)
    torch._dynamo.reset()
    cm = torch.compile(m, fullgraph=True, dynamic=True)
    l_c, g_c = step(cm)
    l_c2, g_c2 = step(cm)  # a second compiled step reuses the graph and the tape registry
    assert torch.equal(l_eager, l_c) and torch.equal(l_c, l_c2)
    for k in g_eager:
        assert torch.equal(g_eager[k], g_c[k]), k
        assert torch.equal(g_c[k], g_c2[k]), k
    import sdpnet_ops
    assert not sdpnet_ops._TAPES  # every tape was consumed by its backward


# --------------------------------------------------------------- compiled DDP (training_tools.py:36-39)
def _ddp_compile_worker(rank, world, port, q, compiled):
    import os
    import torch.distributed as dist
    import torch.nn.functional as F
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        m = _model(ffn_dropout=0.2, attn_dropout=0.2, stochastic_depth_p=[0.1, 0.2]).to("cuda").train()
        # small buckets: several all-reduce buckets per backward, as at full size
        ddp = torch.nn.parallel.DistributedDataParallel(m, bucket_cap_mb=1)
        net = ddp
        if compiled:
            torch._dynamo.reset()
            torch._dynamo.utils.counters.clear()
            net = torch.compile(ddp, dynamic=True)
        g = torch.Generator().manual_seed(100 + rank)
        x = torch.randn(3, 3, 224, 224, generator=g).to("cuda")
        y = torch.randint(0, 10, (3,), generator=g).to("cuda")
        out = []
        for step in range(2):
            m.zero_grad(set_to_none=True)
            torch.manual_seed(7 + step)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits = net(x)
            loss = F.cross_entropy(logits.float(), y, label_smoothing=0.1)
            loss.backward()
            out.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]).cpu().numpy().copy())
        breaks = dict(torch._dynamo.utils.counters["graph_break"]) if compiled else {}
        base = {}
        if compiled:  # the same wrapping of a stock torch module: breaks that DDP itself causes
            torch._dynamo.reset()
            torch._dynamo.utils.counters.clear()
            lin = torch.nn.parallel.DistributedDataParallel(torch.nn.Linear(8, 8).to("cuda"), bucket_cap_mb=1)
            torch.compile(lin, dynamic=True)(torch.randn(4, 8, device="cuda")).sum().backward()
            base = dict(torch._dynamo.utils.counters["graph_break"])
        if rank == 0:
            q.put((out, (breaks, base)))
    finally:
        dist.destroy_process_group()


def _ddp_run(compiled):
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_compile_worker, args=(r, 2, port, q, compiled)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=400)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    return res


@pytest.mark.gpu
def test_compiled_ddp_equals_eager_ddp_bit_for_bit():
    """torch.compile(DDP(model), dynamic=True) as training_tools.py:36-39 builds it, two gloo ranks
    sharing the box's GPU: the per-sub-layer ops give 0 graph breaks and the all-reduced gradients
    of two steps (dropout, drop path, bf16 autocast) equal eager DDP's bit for bit."""
    eager, _ = _ddp_run(False)
    comp, (breaks, base) = _ddp_run(True)
    for a, b in zip(eager, comp):
        assert (a == b).all()
    # no graph break beyond those torch.compile(DDP(nn.Linear)) has on this torch build
    extra = {k: v for k, v in breaks.items() if k not in base}
    assert not extra, "\n".join(extra)
