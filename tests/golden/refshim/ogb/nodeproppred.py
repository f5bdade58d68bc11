class PygNodePropPredDataset:  # import-only stub
    pass


class Evaluator:
    pass
