"""Minimal prototxt -> layer-dict reader for tests (independent of the product's C++ reader)."""
import re


def parse(text):
    text = re.sub(r"#[^\n]*", "", text)
    layers = []
    for body in _blocks(text, "layer"):
        d = {"name": _get(body, "name"), "type": _get(body, "type"),
             "bottom": re.findall(r'bottom:\s*"([^"]+)"', body),
             "top": re.findall(r'top:\s*"([^"]+)"', body)}
        if d["type"] == "Convolution":
            d["num_output"] = int(_get(body, "num_output"))
            d["kernel_size"] = int(_get(body, "kernel_size"))
            d["pad"] = int(_get(body, "pad") or 0)
        elif d["type"] == "Pooling":
            d["kernel_size"] = int(_get(body, "kernel_size"))
            d["stride"] = int(_get(body, "stride") or 1)
        layers.append(d)
    chans = {"image": 3}
    for l in layers:
        if l["type"] == "Convolution":
            l["cin"] = chans[l["bottom"][0]]
            chans[l["top"][0]] = l["num_output"]
        elif l["type"] == "Pooling":
            chans[l["top"][0]] = chans[l["bottom"][0]]
        elif l["type"] == "Concat":
            chans[l["top"][0]] = sum(chans[b] for b in l["bottom"])
    return layers


def _get(body, key):
    m = re.search(key + r':\s*"?([^"\s}]+)"?', body)
    return m.group(1) if m else None


def _blocks(text, key):
    out = []
    for m in re.finditer(r"\b%s\s*\{" % key, text):
        i, depth = m.end(), 1
        while depth:
            depth += {"{": 1, "}": -1}.get(text[i], 0)
            i += 1
        out.append(text[m.end():i - 1])
    return out


def emit(layers):
    """layer dicts -> prototxt text."""
    out = ['name: "test"', 'input: "image"']
    for l in layers:
        s = ['layer {', '  name: "%s"' % l["name"], '  type: "%s"' % l["type"]]
        s += ['  bottom: "%s"' % b for b in l["bottom"]]
        s += ['  top: "%s"' % t for t in l["top"]]
        if l["type"] == "Convolution":
            s.append('  convolution_param { num_output: %d pad: %d kernel_size: %d }'
                     % (l["num_output"], l.get("pad", 1 if l["kernel_size"] == 3 else 0),
                        l["kernel_size"]))
        if l["type"] == "Pooling":
            s.append('  pooling_param { pool: MAX kernel_size: 2 stride: 2 }')
        if l["type"] == "Concat":
            s.append('  concat_param { axis: 1 }')
        s.append('}')
        out += s
    return "\n".join(out) + "\n"
