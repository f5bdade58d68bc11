"""Drop-in replacement for the reference ``layer`` package (layer/__init__.py:1-6): the same six
classes, same constructors / forward signatures / state_dict keys, running on libregnn_hip."""
from layer.REGraphConv import REGraphConv  # noqa: F401
from layer.REGATConv import REGATConv  # noqa: F401
from layer.REMixHopConv import REMixHopConv  # noqa: F401
from layer.RESAGEConv import RESAGEConv  # noqa: F401
from layer.REGATv2Conv import REGATv2Conv  # noqa: F401
from layer.REGINConv import REGINConv  # noqa: F401
