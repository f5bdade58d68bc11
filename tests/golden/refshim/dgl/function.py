"""Message / reduce descriptors (DGL ``dgl.function`` surface used by the reference)."""


class _Msg:
    def __init__(self, kind, a, b, out):
        self.kind, self.a, self.b, self.out = kind, a, b, out


class _Red:
    def __init__(self, kind, msg, out):
        self.kind, self.msg, self.out = kind, msg, out


def u_mul_e(lhs, rhs, out):
    return _Msg("u_mul_e", lhs, rhs, out)


def copy_u(u, out):
    return _Msg("copy_u", u, None, out)


def copy_src(src, out):
    return _Msg("copy_u", src, None, out)


def u_add_v(lhs, rhs, out):
    return _Msg("u_add_v", lhs, rhs, out)


def sum(msg, out):  # noqa: A001 - DGL name
    return _Red("sum", msg, out)


def mean(msg, out):
    return _Red("mean", msg, out)


def max(msg, out):  # noqa: A001 - DGL name
    return _Red("max", msg, out)
