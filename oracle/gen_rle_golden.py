"""TEST INFRASTRUCTURE ONLY -- extracts a small RLE fixture from the reference's own annotation
files (data/endovis18.json, data/endovis18_coco_annotations_val_opened.json; this container
only) into tests/golden/rle_endovis18_sample.json: compressed-RLE strings with the `area` (and,
for the original conversion, `bbox`) that pycocotools computed when the reference wrote them.
The opened file keeps the pre-opening bbox, so only its area is recorded."""
import json
import os

REF = "/root/reference/data"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "rle_endovis18_sample.json")


def main(n=24):
    a = json.load(open(os.path.join(REF, "endovis18.json")))["annotations"]
    b = json.load(open(os.path.join(REF, "endovis18_coco_annotations_val_opened.json")))["annotations"]
    step_a, step_b = max(1, len(a) // n), max(1, len(b) // n)
    out = {"original": [{"segmentation": x["segmentation"], "area": x["area"], "bbox": x["bbox"]} for x in a[::step_a][:n]],
           "opened": [{"segmentation": x["segmentation"], "area": x["area"]} for x in b[::step_b][:n]]}
    with open(OUT, "w") as f:
        json.dump(out, f)
    print(OUT, os.path.getsize(OUT))


if __name__ == "__main__":
    main()
