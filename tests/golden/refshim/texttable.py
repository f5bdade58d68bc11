class Texttable:  # import-only stub
    pass
