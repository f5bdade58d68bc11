class NeighborSampler:  # import-only stub
    pass
