"""Per-node model agent (Scout -> Gopher -> node ConfigMap / node labels)."""
from ome_amd.modelagent.agent import (DELETE, DOWNLOAD, DOWNLOAD_OVERRIDE, Gopher, ModelAgent, NodeConfigMap,
                                      NodeLabeler, Scout, Task, dest_path, model_key)

__all__ = ["ModelAgent", "NodeConfigMap", "NodeLabeler", "Scout", "Gopher", "Task", "model_key", "dest_path",
           "DOWNLOAD", "DOWNLOAD_OVERRIDE", "DELETE"]
