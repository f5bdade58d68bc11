class DGLError(Exception):
    """Raised for invalid graph operations (mirrors dgl.base.DGLError)."""
