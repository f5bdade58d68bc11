def expand_as_pair(input_, g=None):
    """(src, dst) feature pair: tuples pass through, a single tensor serves both sides."""
    if isinstance(input_, tuple):
        return input_
    if g is not None and getattr(g, "is_block", False):
        return input_, input_[:g.number_of_dst_nodes()]
    return input_, input_
