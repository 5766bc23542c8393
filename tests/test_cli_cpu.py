"""omectl against the manager REST API (simulated node)."""
import json

from ome_amd.cli import main as omectl
from ome_amd.manager import Cluster


def test_omectl_roundtrip(tmp_path, capsys):
    cl = Cluster(str(tmp_path / "state"), simulate=True, gpus=8)
    try:
        url = cl.serve_api()
        f = tmp_path / "m.yaml"
        f.write_text(f"""apiVersion: ome.io/v1beta1
kind: ClusterBaseModel
metadata:
  name: tiny
spec:
  vendor: meta
  storage:
    storageUri: random://tiny-llama
    path: {tmp_path}/models/tiny
""")
        assert omectl(["--server", url, "apply", "-f", str(f)]) == 0
        assert "clusterbasemodel/tiny configured" in capsys.readouterr().out
        cl.agent.start()
        cl.step(3)
        assert omectl(["--server", url, "get", "cbm"]) == 0
        out = capsys.readouterr().out
        assert "tiny" in out and "LlamaForCausalLM" in out and "Ready" in out
        assert omectl(["--server", url, "get", "cbm", "tiny", "-o", "json"]) == 0
        assert json.loads(capsys.readouterr().out)["status"]["state"] == "Ready"
        assert omectl(["--server", url, "wait", "cbm", "tiny", "--for", "Ready", "--timeout", "5"]) == 0
        assert omectl(["--server", url, "get", "nodes"]) == 0
        assert "mi355x-node-0" in capsys.readouterr().out
        assert omectl(["--server", url, "delete", "cbm", "tiny"]) == 0
    finally:
        cl.shutdown()
