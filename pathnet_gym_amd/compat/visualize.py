"""``visualize.GraphVisualize`` (ref ``visualize.py:10-118``) -- implemented in ``utils/visualize.py``."""
from ..utils.visualize import GraphVisualize  # noqa: F401
