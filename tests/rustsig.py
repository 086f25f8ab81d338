"""Public-API signatures of Rust source files, for comparing the MI355X drop-in
crates (integration/rust/) with the reference's.

No Rust toolchain exists in the image, so this is a small text parser: it
drops comments and the items under `#[cfg(test)]` / `#[cfg(feature =
"never")]`, then records

  structs   name -> generics, bounds per type parameter
  methods   "Type::name" -> params, return type, the impl block's bounds
  fns       free `pub fn` name -> params, return type, bounds
  macros    `#[macro_export] macro_rules!` names
  enums     name -> variant names
  uses      names re-exported with `pub use`

Whitespace is normalised away around punctuation so that formatting does not
matter; parameter names and types must match exactly.
"""
import re

PUNCT = "<>()[]{},:;&*=+!"


def norm(s: str) -> str:
    s = " ".join(s.split())
    out = []
    for i, ch in enumerate(s):
        if ch == " ":
            prev = out[-1] if out else ""
            nxt = s[i + 1] if i + 1 < len(s) else ""
            if prev in PUNCT or nxt in PUNCT or nxt == "-" or prev == ">":
                continue
        out.append(ch)
    s = "".join(out)
    return s.replace(",)", ")").replace(",>", ">").replace(",}", "}")


def strip_comments(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def _match(src: str, i: int, open_ch: str, close_ch: str) -> int:
    """Index just past the bracket that closes the one at src[i]."""
    assert src[i] == open_ch, (src[i:i + 40], open_ch)
    depth = 0
    while i < len(src):
        c = src[i]
        if c == open_ch:
            depth += 1
        elif c == close_ch:
            depth -= 1
            if depth == 0:
                return i + 1
        i += 1
    raise ValueError("unbalanced")


def _angle_end(src: str, i: int) -> int:
    """Past the `>` closing the generic list at src[i] == '<' (skips `->`)."""
    depth = 0
    while i < len(src):
        c = src[i]
        if c == "<":
            depth += 1
        elif c == ">" and src[i - 1] != "-":
            depth -= 1
            if depth == 0:
                return i + 1
        i += 1
    raise ValueError("unbalanced <>")


def _item_end(src: str, i: int) -> int:
    """End of the item starting at i: its `{...}` body or its `;`."""
    depth = 0
    while i < len(src):
        c = src[i]
        if c in "([":
            depth += 1
        elif c in ")]":
            depth -= 1
        elif c == "{" and depth == 0:
            return _match(src, i, "{", "}")
        elif c == ";" and depth == 0:
            return i + 1
        i += 1
    return len(src)


def drop_cfg_items(src: str, cfgs=("test", 'feature = "never"')) -> str:
    for cfg in cfgs:
        pat = re.compile(r"#\[cfg\(\s*" + re.escape(cfg).replace(r"\ ", r"\s*") + r"\s*\)\]")
        while True:
            m = pat.search(src)
            if not m:
                break
            j = m.end()
            # skip further attributes on the same item
            while True:
                k = len(src[j:]) - len(src[j:].lstrip())
                if src[j + k:j + k + 2] == "#[":
                    j = _match(src, j + k + 1, "[", "]")
                else:
                    break
            src = src[:m.start()] + src[_item_end(src, j):]
    return src


def split_top(s: str, sep=","):
    out, depth, cur = [], 0, ""
    for i, ch in enumerate(s):
        if ch in "(<[{":
            depth += 1
        elif ch in ")]}" or (ch == ">" and (i == 0 or s[i - 1] != "-")):
            depth -= 1
        if ch == sep and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [x.strip() for x in out if x.strip()]


def bounds_of(generics: str, where: str) -> dict:
    """{type param or path: sorted bounds} from `<...>` and a where clause."""
    b = {}
    parts = split_top(generics[1:-1]) if generics else []
    parts += split_top(where)
    for p in parts:
        m = re.match(r"^(.*?[^:]):(?!:)(.*)$", p, flags=re.S)   # first ':' that is not '::'
        if p.startswith("'") or not m:
            continue
        name, bound = m.group(1), m.group(2)
        b.setdefault(norm(name), set()).update(norm(x) for x in split_top(bound, "+"))
    return {k: sorted(v) for k, v in sorted(b.items())}


def _generic_names(generics: str):
    if not generics:
        return []
    return [norm(p.split(":")[0]) for p in split_top(generics[1:-1])]


FN_RE = re.compile(r"\bpub\s+(?:const\s+|unsafe\s+)?fn\s+(\w+)\s*")


def _parse_fn(src: str, m):
    """(name, generics, params, ret, where, end) of the fn whose match is m."""
    i = m.end()
    generics = ""
    if src[i] == "<":
        e = _angle_end(src, i)
        generics, i = src[i:e], e
    while src[i].isspace():
        i += 1
    e = _match(src, i, "(", ")")
    params = [norm(p) for p in split_top(src[i + 1:e - 1])]
    rest_end = _item_end(src, e)
    body_at = src.find("{", e, rest_end) if src[rest_end - 1] == "}" else rest_end - 1
    sig_tail = src[e:body_at]
    ret, where = "", ""
    wm = re.search(r"\bwhere\b", sig_tail)
    if wm:
        where = sig_tail[wm.end():]
        sig_tail = sig_tail[:wm.start()]
    if "->" in sig_tail:
        ret = norm(sig_tail.split("->", 1)[1])
    return m.group(1), generics, params, ret, where, rest_end


def parse(src: str) -> dict:
    src = drop_cfg_items(strip_comments(src))
    api = {"structs": {}, "methods": {}, "fns": {}, "macros": [], "enums": {}, "uses": [], "auto_workspace": []}
    # impl blocks
    impl_spans = []
    for m in re.finditer(r"(?<![\w!])impl\b", src):
        i = m.end()
        while src[i].isspace():
            i += 1
        generics = ""
        if src[i] == "<":
            e = _angle_end(src, i)
            generics, i = src[i:e], e
        body_at = src.index("{", i)
        head = src[i:body_at]
        where = ""
        wm = re.search(r"\bwhere\b", head)
        if wm:
            where, head = head[wm.end():], head[:wm.start()]
        if re.search(r"\bfor\b", head):      # trait impls are not API items here
            impl_spans.append((m.start(), _match(src, body_at, "{", "}")))
            continue
        tname = re.match(r"\s*([\w:]+)", head).group(1).split("::")[-1]
        end = _match(src, body_at, "{", "}")
        impl_spans.append((m.start(), end))
        body = src[body_at + 1:end - 1]
        ib = bounds_of(generics, where)
        for fm in FN_RE.finditer(body):
            name, fg, params, ret, fwhere, _ = _parse_fn(body, fm)
            api["methods"][f"{tname}::{name}"] = {
                "generics": norm(fg), "params": params, "ret": ret,
                "bounds": {**ib, **bounds_of(fg, fwhere)}}
    def outside(pos):
        return all(not (a <= pos < b) for a, b in impl_spans)
    for fm in FN_RE.finditer(src):
        if not outside(fm.start()):
            continue
        name, fg, params, ret, fwhere, _ = _parse_fn(src, fm)
        api["fns"][name] = {"generics": norm(fg), "params": params, "ret": ret, "bounds": bounds_of(fg, fwhere)}
        pre = src[max(0, fm.start() - 200):fm.start()]
        if re.search(r"#\[auto_workspace\]\s*$", pre):
            api["auto_workspace"].append(name)
    for sm in re.finditer(r"\bpub\s+struct\s+(\w+)\s*", src):
        i = sm.end()
        generics = ""
        if src[i] == "<":
            e = _angle_end(src, i)
            generics, i = src[i:e], e
        end = _item_end(src, i)
        body_at = src.find("{", i, end)
        head = src[i:body_at if body_at >= 0 else end]
        where = ""
        wm = re.search(r"\bwhere\b", head)
        if wm:
            where = head[wm.end():]
        api["structs"][sm.group(1)] = {"generics": _generic_names(generics), "bounds": bounds_of(generics, where)}
    for em in re.finditer(r"\bpub\s+enum\s+(\w+)[^{]*\{", src):
        body = src[em.end():_match(src, em.end() - 1, "{", "}") - 1]
        body = re.sub(r"#\[[^\]]*\]", "", body)
        variants = [re.match(r"\s*(\w+)", v).group(1) for v in split_top(body) if re.match(r"\s*\w", v)]
        api["enums"][em.group(1)] = sorted(variants)
    for mm in re.finditer(r"#\[macro_export\][\s\S]{0,200}?macro_rules!\s*(\w+)", src):
        api["macros"].append(mm.group(1))
    api["macros"] = sorted(set(api["macros"]))
    for um in re.finditer(r"\bpub\s+use\s+([^;]+);", src):
        spec = um.group(1)
        if "{" in spec:
            inner = spec[spec.index("{") + 1:spec.rindex("}")]
            names = [x.strip().split(" as ")[-1] for x in inner.split(",") if x.strip()]
        else:
            names = [spec.strip().split("::")[-1].split(" as ")[-1]]
        api["uses"].extend(n.strip() for n in names if n.strip() != "*")
    api["uses"] = sorted(set(api["uses"]))
    for tm in re.finditer(r"\bpub\s+type\s+(\w+)", src):
        api["uses"].append(tm.group(1))
    return api


def merge(*apis) -> dict:
    out = {"structs": {}, "methods": {}, "fns": {}, "macros": [], "enums": {}, "uses": [], "auto_workspace": []}
    for a in apis:
        for k in ("structs", "methods", "fns", "enums"):
            out[k].update(a[k])
        for k in ("macros", "uses", "auto_workspace"):
            out[k] = sorted(set(out[k]) | set(a[k]))
    return out


def expand_auto_workspace(api: dict) -> dict:
    """The `_st` / `_mt` functions `#[auto_workspace]` generates: the same
    signature without the leading workspace parameter
    (ag-cuda-workspace-macro/src/lib.rs:21-51)."""
    for name in api["auto_workspace"]:
        f = api["fns"][name]
        for suffix in ("_st", "_mt"):
            api["fns"][name + suffix] = {**f, "params": f["params"][1:]}
    return api
