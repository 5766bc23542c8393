"""Runtime-args merge / TP-PP override semantics (reference
``pkg/controller/v1beta1/inferenceservice/utils/merging.go:466-525`` MergeArgs /
OverrideArgParam, behaviour pinned by its ``merging_test.go`` cases) plus spec merging."""
import pytest

from ome_amd.controllers.isvc import merging as M

ML = "python3 -m sglang.launch_server \\\n"


def ml(*lines):
    return ["".join(lines[:1]) + "".join(" \\\n" + line for line in lines[1:])]


MERGE_CASES = [
    # multiline (backslash continuation) container args
    (ml("python3 -m sglang.launch_server", "--host=0.0.0.0", "--port=8080", "--enable-metrics", "--log-requests",
        '--model-path="$MODEL_PATH"', "--mem-frac=0.9"), ["--tp-size=4"],
     ml("python3 -m sglang.launch_server", "--host=0.0.0.0", "--port=8080", "--enable-metrics", "--log-requests",
        '--model-path="$MODEL_PATH"', "--mem-frac=0.9", "--tp-size=4")),
    (["python3 -m server"], [], ["python3 -m server"]),
    ([], ["--tp-size=4"], ["--tp-size=4"]),
    (["python3 -m server"], ["--debug"], ["python3 -m server", "--debug"]),
    (ml("python3 -m sglang.launch_server", "--host=0.0.0.0"), ["--tp-size=4", "--pp-size=2"],
     ml("python3 -m sglang.launch_server", "--host=0.0.0.0", "--tp-size=4", "--pp-size=2")),
    (["python3 -m sglang.launch_server\n--host=0.0.0.0\n--port=8080"], ["--tp-size=4"],
     ["python3 -m sglang.launch_server \\\n--host=0.0.0.0 \\\n--port=8080 \\\n--tp-size=4"]),
    # list format
    (["--tp-size=4", "--port=8080"], ["--tp-size=8"], ["--tp-size=8", "--port=8080"]),
    (["--tp-size=4", "--port=8080"], ["--host=0.0.0.0"], ["--tp-size=4", "--port=8080", "--host=0.0.0.0"]),
    (["--tp-size=4", "--pp-size=2", "--port=8080"], ["--tp-size=8", "--pp-size=4", "--debug"],
     ["--tp-size=8", "--pp-size=4", "--port=8080", "--debug"]),
    (["--tp-size=4", "--port=8080"], ["--tp-size=4"], ["--tp-size=4", "--port=8080"]),
    (["--tp-size", "4", "--port", "8080"], ["--tp-size", "8"], ["--tp-size", "8", "--port", "8080"]),
    (["--tp-size=4", "--port", "8080"], ["--tp-size=8", "--host=0.0.0.0"],
     ["--tp-size=8", "--port", "8080", "--host=0.0.0.0"]),
    (["python3", "-m", "server", "--port=8080"], ["--debug"], ["python3", "-m", "server", "--port=8080", "--debug"]),
    ([], [], []),
    (None, None, []),
    (ml("python3 -m server", "--port=8080"), ["  --tp-size=4  "], ml("python3 -m server", "--port=8080", "--tp-size=4")),
    # union semantics
    (ml("python3 -m server", "--Enable-Metrics"), ["--enable-metrics"],
     ml("python3 -m server", "--Enable-Metrics", "--enable-metrics")),
    (ml("python3 -m server", "--tp-size=4", "--port=8080"), ["--tp-size=8", "--host=0.0.0.0"],
     ml("python3 -m server", "--tp-size=8", "--port=8080", "--host=0.0.0.0")),
    (ml("python3 -m server", "--tp-size 4", "--port 8080"), ["--tp-size 8", "--host 0.0.0.0"],
     ml("python3 -m server", "--tp-size 8", "--port 8080", "--host 0.0.0.0")),
    (ml("python3 -m server", "--enable-metrics", "--port=8080"), ["--enable-metrics", "--debug"],
     ml("python3 -m server", "--enable-metrics", "--port=8080", "--debug")),
    (ml("python3 -m server", "--tp-size=4", "--pp-size=2", "--port=8080"), ["--tp-size=8", "--pp-size=4", "--new-flag"],
     ml("python3 -m server", "--tp-size=8", "--pp-size=4", "--port=8080", "--new-flag")),
]


@pytest.mark.parametrize("base,override,want", MERGE_CASES)
def test_merge_args(base, override, want):
    assert M.merge_args(base, override) == want


OVERRIDE_CASES = [
    (ml("python3 -m sglang.launch_server", "--host=0.0.0.0", "--tp-size=4", "--mem-frac=0.9"), "--tp-size", 8,
     ml("python3 -m sglang.launch_server", "--host=0.0.0.0", "--tp-size=8", "--mem-frac=0.9"), True),
    (ml("python3 -m server", "--tp-size 4", "--mem-frac=0.9"), "--tp-size", 8,
     ml("python3 -m server", "--tp-size=8", "--mem-frac=0.9"), True),
    (ml("python3 -m server", "--host=0.0.0.0"), "--tp-size", 8, ml("python3 -m server", "--host=0.0.0.0"), False),
    ([], "--tp-size", 8, [], False),
    (ml("python3 -m server", "--pp-size=2", "--tp-size=4"), "--pp-size", 4,
     ml("python3 -m server", "--pp-size=4", "--tp-size=4"), True),
    (ml("python3 -m server", "--tensor-parallel-size=4"), "--tensor-parallel-size", 8,
     ml("python3 -m server", "--tensor-parallel-size=8"), True),
    (["--tp-size=4", "--port=8080"], "--tp-size", 8, ["--tp-size=8", "--port=8080"], True),
    (["--tp-size", "4", "--port", "8080"], "--tp-size", 8, ["--tp-size", "8", "--port", "8080"], True),
    (["--port=8080", "--host=0.0.0.0"], "--tp-size", 8, ["--port=8080", "--host=0.0.0.0"], False),
    (["--port=8080", "--tp-size"], "--tp-size", 8, ["--port=8080", "--tp-size"], False),
    (["python3", "-m", "server", "--tp-size=4"], "--tp-size", 8, ["python3", "-m", "server", "--tp-size=8"], True),
    (["python3", "-m", "server", "--tp-size", "4"], "--tp-size", 8, ["python3", "-m", "server", "--tp-size", "8"],
     True),
]


@pytest.mark.parametrize("args,key,value,want,found", OVERRIDE_CASES)
def test_override_arg(args, key, value, want, found):
    got, ok = M.override_arg(args, key, value)
    assert ok == found and got == want


def test_override_param_prefers_args_then_command_and_aliases():
    c = {"command": ["python3", "-m", "sglang.launch_server", "--tp", "2"], "args": ["--port=8080"]}
    assert M.override_param(c, M.TP_ALIASES, 8)
    assert c["command"][-1] == "8" and c["args"] == ["--port=8080"]
    c = {"args": ["--tensor-parallel-size=2"]}
    assert M.override_param(c, M.TP_ALIASES, 4) and c["args"] == ["--tensor-parallel-size=4"]
    assert not M.override_param({"args": ["--port=1"]}, M.PP_ALIASES, 2)


def test_strategic_merge_containers_by_name_and_isvc_wins():
    base = {"containers": [{"name": "ome-container", "image": "a", "env": [{"name": "X", "value": "1"}]}],
            "nodeSelector": {"a": "1"}}
    over = {"containers": [{"name": "ome-container", "image": "b", "env": [{"name": "Y", "value": "2"}]}],
            "nodeSelector": {"b": "2"}}
    out = M.strategic_merge(base, over)
    c = out["containers"][0]
    assert c["image"] == "b"
    assert {e["name"] for e in c["env"]} == {"X", "Y"}
    assert out["nodeSelector"] == {"a": "1", "b": "2"}


def test_replace_placeholders():
    c = {"args": ["--served-model-name={{.Name}}", "--ns={{.Namespace}}"], "env": [{"name": "A", "value": "{{.Name}}"}]}
    out = M.replace_placeholders(c, {"name": "isvc-a", "namespace": "team"})
    assert out["args"] == ["--served-model-name=isvc-a", "--ns=team"]
    assert out["env"][0]["value"] == "isvc-a"


def test_gpu_count_and_env_helpers():
    c = {"resources": {"limits": {"amd.com/gpu": "8"}}}
    assert M.gpu_count(c) == 8
    assert M.gpu_count({"resources": {"requests": {"nvidia.com/gpu": 4}}}) == 4
    M.set_env(c, "A", "1")
    M.set_env(c, "A", "2", overwrite=False)
    assert M.get_env(c, "A") == "1"
    M.set_env(c, "A", "3")
    assert M.get_env(c, "A") == "3"
