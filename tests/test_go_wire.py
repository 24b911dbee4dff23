"""The Go binding's wire constants against the C-ABI header (no Go toolchain
here, so the cgo package is never compiled: these values are cross-checked
as text).  Fails on any drift:

* message type codes: go/api/authen-batch.go AuthenRequest.. vs
  include/minbft_gpu.h enum mbft_msg_type;
* stage codes: go/gpuauth/messages.go st* vs enum mbft_stage;
* roles: the reference's api/api.go (ReplicaAuthen = 1 + iota, USIGAuthen,
  ClientAuthen) vs enum mbft_role, and the binding's roleByte maps only those
  three to themselves (anything else -> 0, MBFT_UNKNOWN_ROLE);
* statuses: every MBFT_* status the Go error mapping names exists in enum
  mbft_status, and every status has a case;
* the flat record: every field of struct mbft_msg_rec is written by the Go
  marshal (go/gpuauth/messages.go), and the header's field order matches the
  Python dtype the tests use (minbft_amd/_lib.py).
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _read(*p):
    with open(os.path.join(ROOT, *p)) as f:
        return f.read()


def _enum(txt, name):
    m = re.search(r"enum\s+" + name + r"\s*\{(.*?)\}", txt, re.S)
    assert m, name
    body = re.sub(r"/\*.*?\*/", "", m.group(1), flags=re.S)
    out = {}
    for k, v in re.findall(r"(MBFT_[A-Z_0-9]+)\s*=\s*(-?\d+)", body):
        out[k] = int(v)
    return out


def _go_consts(txt, names):
    out = {}
    for nm in names:
        m = re.search(r"\b" + nm + r"\s+(?:uint32\s+)?=\s*(\d+)", txt)
        assert m, nm
        out[nm] = int(m.group(1))
    return out


def test_message_type_codes():
    hdr = _enum(_read("include", "minbft_gpu.h"), "mbft_msg_type")
    go = _go_consts(_read("go", "api", "authen-batch.go"),
                    ["AuthenRequest", "AuthenReply", "AuthenPrepare", "AuthenCommit", "AuthenReqViewChange"])
    assert go == {"AuthenRequest": hdr["MBFT_MSG_REQUEST"], "AuthenReply": hdr["MBFT_MSG_REPLY"],
                  "AuthenPrepare": hdr["MBFT_MSG_PREPARE"], "AuthenCommit": hdr["MBFT_MSG_COMMIT"],
                  "AuthenReqViewChange": hdr["MBFT_MSG_REQ_VIEW_CHANGE"]}


def test_stage_codes():
    hdr = _enum(_read("include", "minbft_gpu.h"), "mbft_stage")
    pairs = {"stRequestSig": "MBFT_ST_REQUEST_SIG", "stNotPrimary": "MBFT_ST_NOT_PRIMARY",
             "stPrepareUI": "MBFT_ST_PREPARE_UI", "stCommitFromPrimary": "MBFT_ST_COMMIT_FROM_PRIMARY",
             "stCommitUI": "MBFT_ST_COMMIT_UI", "stNotImplemented": "MBFT_ST_NOT_IMPLEMENTED",
             "stUnknownType": "MBFT_ST_UNKNOWN_TYPE", "stReplySig": "MBFT_ST_REPLY_SIG",
             "stReplyClientID": "MBFT_ST_REPLY_CLIENT_ID"}
    go_txt = _read("go", "gpuauth", "messages.go") + "\n" + _read("go", "gpuauth", "replies.go")
    go = _go_consts(go_txt, list(pairs))
    for g, h in pairs.items():
        assert go[g] == hdr[h], (g, go[g], h, hdr[h])
    # every st* constant the Go files define is one of the checked ones
    defined = set(re.findall(r"^\s*(st[A-Z][A-Za-z]+)\s*=", go_txt, re.M))
    assert defined == set(pairs), defined ^ set(pairs)


def test_roles_and_role_byte():
    hdr = _enum(_read("include", "minbft_gpu.h"), "mbft_role")
    ref = os.path.join("/root/reference", "api", "api.go")
    # the reference (study only; absent on the GPU box): 1 + iota in this order
    if os.path.exists(ref):
        with open(ref) as f:
            txt = f.read()
        block = re.search(r"ReplicaAuthen AuthenticationRole = 1 \+ iota(.*?)\n\)", txt, re.S).group(1)
        order = ["ReplicaAuthen"] + re.findall(r"^\s*(USIGAuthen|ClientAuthen)\s*$", block, re.M)
        assert order == ["ReplicaAuthen", "USIGAuthen", "ClientAuthen"]
    assert hdr == {"MBFT_ROLE_REPLICA": 1, "MBFT_ROLE_USIG": 2, "MBFT_ROLE_CLIENT": 3}
    go = _read("go", "gpuauth", "gpuauth.go")
    fn = re.search(r"func roleByte\(r api\.AuthenticationRole\) byte \{(.*?)\n\}", go, re.S)
    assert fn, "roleByte missing"
    body = fn.group(1)
    assert re.search(r"case api\.ReplicaAuthen, api\.USIGAuthen, api\.ClientAuthen:\s*return byte\(r\)", body)
    assert re.search(r"return 0\s*$", body.strip())
    # no call path narrows a role by conversion: every role the binding hands
    # the library goes through roleByte (registration skips schemeless roles)
    for f in ("gpuauth.go", "keys.go", "messages.go"):
        t = _read("go", "gpuauth", f)
        assert not re.search(r"byte\((?:c\.)?[Rr]ole\)", t.replace("return byte(r)", "")), f
        for m in re.finditer(r"C\.uint32_t\(((?:c\.)?[Rr]ole)\)", t):
            line = t[:m.start()].count("\n") + 1
            ctx = t[max(0, m.start() - 2000):m.start()]
            assert "roleByte(role) == 0" in ctx or "roleByte" in t.splitlines()[line - 1], (f, line)


def test_status_cases():
    hdr = _enum(_read("include", "minbft_gpu.h"), "mbft_status")
    go = _read("go", "gpuauth", "errors.go")
    named = set(re.findall(r"C\.(MBFT_[A-Z_]+)", go))
    assert named <= set(hdr) | set(_enum(_read("include", "minbft_gpu.h"), "mbft_err")), named - set(hdr)
    cases = set(re.findall(r"case C\.(MBFT_[A-Z_]+)", go))
    # ZERO_COUNTER is a core-level check (usig-ui.go:65-67) the message errors map
    missing = set(hdr) - cases - {"MBFT_ZERO_COUNTER"}
    assert not missing, missing
    assert "MBFT_ZERO_COUNTER" in _read("go", "gpuauth", "messages.go")


def test_msg_rec_fields():
    hdr = _read("include", "minbft_gpu.h")
    body = re.search(r"typedef struct mbft_msg_rec \{(.*?)\} mbft_msg_rec;", hdr, re.S).group(1)
    fields = re.findall(r"uint(?:32|64)_t\s+([a-z_]+);", body)
    from minbft_amd._lib import MSG_REC_DTYPE_FIELDS
    assert fields == [f for f, _ in MSG_REC_DTYPE_FIELDS]
    widths = re.findall(r"uint(32|64)_t\s+[a-z_]+;", body)
    assert [{"32": "<u4", "64": "<u8"}[w] for w in widths] == [t for _, t in MSG_REC_DTYPE_FIELDS]
    go = _read("go", "gpuauth", "messages.go")
    for f in fields:
        name = "_type" if f == "type" else f
        assert re.search(r"r\." + name + r"\b", go), f
