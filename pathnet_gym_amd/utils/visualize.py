"""Path-graph visualiser (reference ``visualize.py:10-118``).

Same picture as the reference: an L x M grid of module nodes at
(10*layer, 10*module); every genotype adds edges between the active modules
of consecutive layers, node size and edge width grow with re-use, and the
frozen path is drawn in its own colour and width (red for task 1, green for
task 2 in the reference, ``doom_pathnet.py:276``).  Differences: headless
(matplotlib Agg, no ``pylab.ion``/``waitforbuttonpress``), PNGs go to a
caller-chosen directory, and the networkx 1.x ``graph.node`` API is not used.
"""
from __future__ import annotations

import os
import time
from typing import List, Optional, Sequence


class GraphVisualize:
    node_size_add = 1.5
    init_node_size = 0.1
    edge_weight_add = 0.1
    init_edge_weight = 0.0
    fixed_weight = 6.4

    def __init__(self, modules: Sequence[int], vis: bool = True, out_dir: str = "./data/graphs"):
        import networkx as nx
        self.nx = nx
        self.vis = vis
        self.out_dir = out_dir
        self.graph = nx.Graph()
        self.node_ids = {}
        self.fixed_path: List[List[int]] = [[] for _ in modules]
        self.fixed_color = None
        n = 0
        for layer, m in enumerate(modules):
            for j in range(m):
                self.graph.add_node(n, Position=(10 * layer, 10 * j), size=self.init_node_size)
                self.node_ids[(layer, j)] = n
                n += 1

    def set_fixed(self, path, color: str):
        self.fixed_color = color
        self.fixed_path = [[self.node_ids[(l, int(j))] for j in layer] for l, layer in enumerate(path)]

    def reset(self):
        for _, d in self.graph.nodes(data=True):
            d["size"] = self.init_node_size
        self.graph.remove_edges_from(list(self.graph.edges()))

    def _add_genes(self, genes, color):
        g = self.graph
        for gene in genes:
            for layer in range(len(gene) - 1):
                for a in gene[layer]:
                    for b in gene[layer + 1]:
                        u, v = self.node_ids[(layer, int(a))], self.node_ids[(layer + 1, int(b))]
                        if g.has_edge(u, v):
                            g.nodes[u]["size"] += self.node_size_add
                            g.nodes[v]["size"] += self.node_size_add
                            g[u][v]["weight"] += self.edge_weight_add
                            g[u][v]["color"] = color
                        else:
                            g.add_edge(u, v, color=color, weight=self.init_edge_weight)
        for layer in range(len(self.fixed_path) - 1):
            for u in self.fixed_path[layer]:
                for v in self.fixed_path[layer + 1]:
                    g.add_edge(u, v, color=self.fixed_color, weight=self.fixed_weight)

    def show(self, genes, color: str = "m", filename: Optional[str] = None) -> Optional[str]:
        """Draw the population (list of decoded paths) and save a PNG (visualize.py:90-100)."""
        if not self.vis:
            return None
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        self.reset()
        self._add_genes(genes, color)
        nx = self.nx
        fig = plt.figure(figsize=(6, 6))
        pos = nx.get_node_attributes(self.graph, "Position")
        sizes = [d["size"] for _, d in self.graph.nodes(data=True)]
        nx.draw_networkx_nodes(self.graph, pos=pos, node_color="g", node_size=sizes, node_shape="s")
        edges = list(self.graph.edges())
        if edges:
            nx.draw_networkx_edges(self.graph, pos=pos, edgelist=edges,
                                   edge_color=[self.graph[u][v]["color"] for u, v in edges],
                                   width=[self.graph[u][v]["weight"] for u, v in edges])
        plt.axis("off")
        if filename is None:
            os.makedirs(self.out_dir, exist_ok=True)
            filename = os.path.join(self.out_dir, f"Graph{time.time()}.png")
        else:
            os.makedirs(os.path.dirname(os.path.abspath(filename)), exist_ok=True)
        fig.savefig(filename, format="PNG")
        plt.close(fig)
        return filename

    def waitForButtonPress(self):      # reference API; headless no-op
        return None
