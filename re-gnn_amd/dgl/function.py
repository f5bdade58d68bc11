"""Built-in message / reduce descriptors (dgl.function surface used by RE-GNN)."""
import builtins


class MessageFunc:
    def __init__(self, kind, lhs, rhs, out):
        self.kind, self.lhs, self.rhs, self.out = kind, lhs, rhs, out

    def __repr__(self):
        return f"{self.kind}({self.lhs}, {self.rhs} -> {self.out})"


class ReduceFunc:
    def __init__(self, kind, msg, out):
        self.kind, self.msg, self.out = kind, msg, out


def u_mul_e(lhs_field, rhs_field, out):
    return MessageFunc("u_mul_e", lhs_field, rhs_field, out)


def copy_u(u, out):
    return MessageFunc("copy_u", u, None, out)


copy_src = copy_u


def u_add_v(lhs_field, rhs_field, out):
    return MessageFunc("u_add_v", lhs_field, rhs_field, out)


def sum(msg, out):  # noqa: A001 - DGL name
    return ReduceFunc("sum", msg, out)


def mean(msg, out):
    return ReduceFunc("mean", msg, out)


def max(msg, out):  # noqa: A001 - DGL name
    return ReduceFunc("max", msg, out)


_ = builtins
