def group_hetero_graph(*a, **k):
    raise NotImplementedError
