"""Data-analysis agent (reference: /root/reference/community/data-analysis-agent): query understanding, sandboxed
pandas computation, declarative plots (validated spec -> data + Vega-Lite), reasoning with separated thinking, and
dataset insights."""
from .agent import DataAnalysisAgent, plot_data, split_thinking, wants_plot  # noqa: F401
