"""The in-place accumulation check reads each leaf's AccumulateGrad node off the backward node
(``ctx.next_functions``) instead of ``get_gradient_edge`` (host time per backward).  The mapping from
input index to ``next_functions`` position must skip non-tensor inputs and give exactly the nodes
``get_gradient_edge`` gives, so ``_will_engine_execute_node`` answers the same question (CPU test)."""
import torch
from torch.autograd.graph import get_gradient_edge

import diff_gaussian_rasterization as D


def test_input_nodes_match_gradient_edges():
    a = torch.zeros(3, requires_grad=True)
    b = torch.zeros(3)                       # tensor without grad: (None, 0) edge
    c = torch.zeros(2, 3, requires_grad=True)
    seen = {}

    class F(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, none_arg, y, z, settings):
            ctx.tensor_pos = D._tensor_positions((x, none_arg, y, z))
            return x.sum() + z.sum()

        @staticmethod
        def backward(ctx, g):
            nodes = D._input_nodes(ctx, (0, 1, 2, 3))
            seen["nodes"] = nodes
            seen["will"] = [D._engine_accumulates(t, n) for t, n in ((a, nodes[0]), (c, nodes[3]))]
            seen["ref"] = [get_gradient_edge(a).node, get_gradient_edge(c).node]
            return g * torch.ones(3), None, None, g * torch.ones(2, 3), None

    F.apply(a, None, b, c, "settings").backward()
    nodes = seen["nodes"]
    assert nodes[0] is seen["ref"][0] and nodes[3] is seen["ref"][1]
    assert nodes[1] is None and nodes[2] is None  # a None input, a tensor that needs no grad
    assert seen["will"] == [True, True]


def test_inputs_subset_is_respected():
    a = torch.zeros(3, requires_grad=True)
    c = torch.zeros(3, requires_grad=True)
    seen = {}

    class F(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, y):
            ctx.tensor_pos = D._tensor_positions((x, y))
            return (x * y).sum()

        @staticmethod
        def backward(ctx, g):
            n = D._input_nodes(ctx, (0, 1))
            seen["will"] = [D._engine_accumulates(a, n[0]), D._engine_accumulates(c, n[1])]
            return g * torch.ones(3), g * torch.ones(3)

    F.apply(a, c).backward(inputs=[c])  # only c's AccumulateGrad runs
    assert seen["will"] == [False, True]


def test_fresh_targets_resolve_at_the_flush():
    """Deferred targets of leaves without .grad (D._Fresh): the flush allocates the gradient and the
    first launch overwrites it; a later launch of the same flush adds into it; a .grad that autograd
    set meanwhile is added into in place, or -- in a form the kernel cannot write -- through a
    temporary added afterwards (CPU test of the bookkeeping)."""
    created, post = set(), []
    a = torch.zeros(4, 3, requires_grad=True)
    g, ow = D._fresh_target(D._Fresh(a), created, post)
    assert ow and g is a.grad and g.shape == a.shape and g.is_contiguous()
    created.discard(id(a))  # the first launch wrote it
    g2, ow2 = D._fresh_target(D._Fresh(a), created, post)
    assert g2 is g and not ow2 and not post
    b = torch.zeros(4, 3, requires_grad=True)
    b.grad = torch.ones(4, 3)  # set by AccumulateGrad during the pass
    gb, owb = D._fresh_target(D._Fresh(b), created, post)
    assert gb is b.grad and not owb and not post
    c = torch.zeros(4, 3, requires_grad=True)
    c.grad = torch.ones(3, 4).t()  # non-contiguous: a temporary, added after the launch
    gc, owc = D._fresh_target(D._Fresh(c), created, post)
    assert gc is not c.grad and not owc and post == [(c, gc)] and not gc.any()
    t = torch.ones(4, 3)
    assert D._fresh_target(t, created, post) == (t, False)  # an existing target passes through
    assert D._fresh_target(None, created, post) == (None, False)
