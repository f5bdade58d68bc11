from . import nodeproppred  # noqa: F401
