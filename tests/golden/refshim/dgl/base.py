class DGLError(Exception):
    pass
