"""Static HTML report cards (the `@card` + Markdown/Table/Image/Artifact components used by the
eval flow's error-analysis card, R/eval_flow.py:96-139)."""
from __future__ import annotations

import base64
import html
import io
import os


class Markdown:
    def __init__(self, text: str):
        self.text = text

    def render(self) -> str:
        out = []
        for line in self.text.splitlines():
            s = line.strip()
            n = len(s) - len(s.lstrip("#"))
            if 0 < n <= 6 and s[n:n + 1] == " ":
                out.append(f"<h{n}>{html.escape(s[n + 1:])}</h{n}>")
            elif s:
                out.append(f"<p>{html.escape(s)}</p>")
        return "\n".join(out)


class Image:
    def __init__(self, png_bytes: bytes, label: str | None = None):
        self.png, self.label = png_bytes, label

    @classmethod
    def from_matplotlib(cls, fig, label: str | None = None) -> "Image":
        buf = io.BytesIO()
        fig.savefig(buf, format="png", bbox_inches="tight")
        return cls(buf.getvalue(), label)

    @classmethod
    def from_pil_image(cls, img, label=None):
        buf = io.BytesIO()
        img.save(buf, format="PNG")
        return cls(buf.getvalue(), label)

    def render(self) -> str:
        b64 = base64.b64encode(self.png).decode()
        cap = f"<figcaption>{html.escape(self.label)}</figcaption>" if self.label else ""
        return f'<figure><img src="data:image/png;base64,{b64}"/>{cap}</figure>'


class Artifact:
    def __init__(self, obj, name: str | None = None):
        self.obj, self.name = obj, name

    def render(self) -> str:
        return f"<pre>{html.escape((self.name + ': ') if self.name else '')}{html.escape(repr(self.obj))}</pre>"


class Table:
    def __init__(self, data=None, headers=None):
        self.data, self.headers = data or [], headers or []

    def render(self) -> str:
        def cell(c):
            if hasattr(c, "render"):
                return c.render()
            return html.escape(str(c))

        head = "".join(f"<th>{html.escape(str(h))}</th>" for h in self.headers)
        rows = "".join("<tr>" + "".join(f"<td>{cell(c)}</td>" for c in r) + "</tr>" for r in self.data)
        return f"<table><thead><tr>{head}</tr></thead><tbody>{rows}</tbody></table>"


class Card:
    def __init__(self, card_id: str, card_type: str = "blank"):
        self.id, self.type = card_id, card_type
        self.components: list = []

    def append(self, comp):
        self.components.append(comp)

    def extend(self, comps):
        self.components.extend(comps)

    def clear(self):
        self.components.clear()

    def render(self, title: str) -> str:
        body = "\n".join(c.render() if hasattr(c, "render") else html.escape(str(c)) for c in self.components)
        css = ("body{font-family:sans-serif;margin:2em} table{border-collapse:collapse} "
               "td,th{border:1px solid #ccc;padding:4px;vertical-align:middle} img{max-width:360px}")
        return (f"<!doctype html><html><head><meta charset='utf-8'><title>{html.escape(title)}</title>"
                f"<style>{css}</style></head><body><h1>{html.escape(title)}</h1>{body}</body></html>")

    def save(self, directory: str, title: str) -> str:
        os.makedirs(directory, exist_ok=True)
        p = os.path.join(directory, f"{self.id}.html")
        with open(p, "w") as f:
            f.write(self.render(title))
        return p


class CardRegistry(dict):
    """`current.card['id']` -> Card (created on first access)."""

    def __missing__(self, key):
        c = Card(key)
        self[key] = c
        return c

    def append(self, comp):  # default card
        self["default"].append(comp)


def error_analysis_components(predictions, misclassified, labels_map: dict, n_samples: int = 50,
                              image_shape=(28, 28)) -> list:
    """The eval flow's error-analysis card (R/eval_flow.py:96-139) as card components: a
    "Misclassifications X out of Y" heading and a table of up to `n_samples` misclassified rows
    (deterministic sample) with the input image, true / predicted label and a logits bar chart.
    `predictions` / `misclassified` are DataFrames with features, labels, predicted_values and
    logits columns.  Renders with matplotlib's Agg backend (no display needed)."""
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    total, wrong = predictions.shape[0], misclassified.shape[0]
    picked = misclassified.sample(min(n_samples, wrong), random_state=0) if wrong else misclassified
    names = list(labels_map.values())

    def image_of(features):
        fig, ax = plt.subplots()
        ax.imshow(features.reshape(*image_shape), cmap="gray")
        ax.axis("off")
        img = Image.from_matplotlib(fig)
        plt.close(fig)
        return img

    def logits_chart(logits):
        fig, ax = plt.subplots(figsize=(6, 4))
        bars = ax.barh(names, logits)
        ax.set(title="Logits", xlabel="Value", ylabel="Category")
        ax.spines[["right", "top"]].set_visible(False)
        for bar, v in zip(bars, logits):
            ax.text(v, bar.get_y() + bar.get_height() / 2, f"{v:.2f}", va="center")
        fig.tight_layout()
        img = Image.from_matplotlib(fig)
        plt.close(fig)
        return img

    rows = [[image_of(r.features), labels_map[int(r.labels)], labels_map[int(r.predicted_values)], logits_chart(r.logits)]
            for _, r in picked.iterrows()]
    return [Markdown(f"### Misclassifications {wrong} out of {total}"),
            Table(headers=["Image", "True label", "Predicted label", "Logits"], data=rows)]
