"""torch.ops.maleague.* (maleague/ops.py): the stand-alone hot-path ops registered as PyTorch custom operators.
CPU: registration and the fake (meta) implementations' shapes -- what torch.compile traces with. GPU: each op equals
its module's previous direct C-ABI path, passes torch.library.opcheck, and compiles into a full graph."""
import pytest
import torch


def test_ops_registered_with_fake_shapes():
    import maleague  # noqa: F401  (registers the ops)
    from torch._subclasses.fake_tensor import FakeTensorMode
    from maleague.ops import OPS
    for name in OPS:
        assert hasattr(torch.ops.maleague, name), name
    with FakeTensorMode():
        q, h = torch.ops.maleague.agent_forward(torch.empty(10), torch.empty(40, 100), torch.empty(40, 64),
                                                [80, 15, 5, 64, 100, 1, 1])
        assert q.shape == (40, 15) and h.shape == (40, 64)
        a, g = torch.ops.maleague.select_actions(torch.empty(8, 5, 15), torch.empty(8, 5, 15, dtype=torch.int32),
                                                 torch.empty(8, dtype=torch.int64), torch.empty(8, dtype=torch.int32),
                                                 0, 0.1)
        assert a.shape == (8, 5) and a.dtype == torch.int64 and g.dtype == torch.int64
        y = torch.ops.maleague.refil_attention(torch.empty(192, 64), torch.empty(64, 64), torch.empty(64),
                                               torch.empty(6, 16, 64), torch.empty(6, 8, 16, dtype=torch.uint8),
                                               torch.empty(6, 8, dtype=torch.uint8), 4)
        assert y.shape == (6, 8, 64)
        qs, hs = torch.ops.maleague.refil_agent_step(torch.empty(10), torch.empty(6, 16, 29),
                                                     torch.empty(6, 16, 16, dtype=torch.uint8),
                                                     torch.empty(6, 16, dtype=torch.uint8), torch.empty(6, 8, 64),
                                                     [8, 16, 8, 21, 1, 64, 4, 64])
        assert qs.shape == (6, 8, 21) and hs.shape == (6, 8, 64)
        out = torch.ops.maleague.qmix_forward([torch.empty(1)] * 14, torch.empty(12, 5), torch.empty(12, 60),
                                              [5, 60, 32, 64, 2])
        assert out.shape == (12,)


def test_ops_refuse_host_tensors():
    import maleague  # noqa: F401
    from maleague._native import NativeError
    with pytest.raises((NativeError, RuntimeError)):
        torch.ops.maleague.agent_forward(torch.zeros(10), torch.zeros(4, 100), torch.zeros(4, 64),
                                         [80, 15, 5, 64, 100, 1, 1])


@pytest.mark.gpu
def test_agent_forward_op_matches_and_compiles(device):
    """DRQNAgentNetwork.forward through torch.ops.maleague.agent_forward == the golden DRQN step (drqn_agent.py:29-35);
    opcheck passes; torch.compile(fullgraph=True) of a function around the op runs it as one node."""
    import numpy as np
    from helpers import qmix_args
    from maleague.modules.agents.drqn_agent import DRQNAgentNetwork
    from conftest import GOLDEN
    d = np.load(f"{GOLDEN}/drqn_step.npz")
    ag = DRQNAgentNetwork(100, qmix_args(n_agents=5, n_actions=15))
    ag.load_state_dict({k[2:]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith("p.")})
    x, h = torch.from_numpy(d["inputs"]).to(device), torch.from_numpy(d["hidden"]).to(device)
    q, h2 = ag(x, h)
    np.testing.assert_allclose(q.cpu().numpy(), d["q"], atol=1e-4, rtol=0)
    np.testing.assert_allclose(h2.cpu().numpy(), d["h"], atol=1e-4, rtol=0)
    from maleague.ops import struct_fields
    dims = struct_fields(ag.dims())
    torch.library.opcheck(torch.ops.maleague.agent_forward.default, (ag.packed(), x, h.contiguous(), dims),
                          test_utils=("test_schema", "test_faketensor"))

    def f(P, xx, hh):
        qq, hn = torch.ops.maleague.agent_forward(P, xx, hh, dims)
        return qq.argmax(-1), hn

    cf = torch.compile(f, fullgraph=True, backend="eager")
    a1, hn1 = cf(ag.packed(), x, h.contiguous())
    assert torch.equal(a1, q.argmax(-1)) and torch.equal(hn1, h2)
