"""TEST-ONLY MessagePassing (source_to_target: x_j = x[0][edge_index[0]], aggregate at
edge_index[1] with dim_size = x[1].size(0), then ``update``) for the golden generator."""
import inspect

import torch

from torch_scatter import scatter


class MessagePassing(torch.nn.Module):
    def __init__(self, aggr="add", **kwargs):
        super().__init__()
        self.aggr = {"add": "sum"}.get(aggr, aggr)

    def propagate(self, edge_index, size=None, **kwargs):
        x = kwargs.get("x")
        params = inspect.signature(self.message).parameters
        margs = {}
        for name in params:
            if name == "x_j":
                margs[name] = (x[0] if isinstance(x, tuple) else x)[edge_index[0]]
            elif name == "x_i":
                margs[name] = (x[1] if isinstance(x, tuple) else x)[edge_index[1]]
            elif name == "index":
                margs[name] = edge_index[1]
            else:
                margs[name] = kwargs[name]
        msg = self.message(**margs)
        n = (x[1] if isinstance(x, tuple) else x).size(0)
        out = scatter(msg, edge_index[1], 0, dim_size=n, reduce=self.aggr)
        return self.update(out)

    def update(self, aggr_out):
        return aggr_out


class GATv2Conv:  # import-only stub
    pass
