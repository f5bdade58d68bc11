class SparseTensor:  # import-only stub
    pass
