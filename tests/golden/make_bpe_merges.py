"""Write a small CLIP-format BPE merges file for the tokenizer fixtures (run in the build container).

    python tests/golden/make_bpe_merges.py

CLIP's own `bpe_simple_vocab_16e6.txt.gz` is not in this image (no network), so the tokenizer is pinned
on a merges file of the same format learned here: byte-level symbols (clip/simple_tokenizer.py:15-35),
an end-of-word marker `</w>` on each word's last symbol, one "a b" merge per line after a version
header.  The corpus is remote-sensing class names (the PatternNet / UCMerced / EuroSAT label sets the
federated clients use), caption-style sentences and a little general English with digits, punctuation,
contractions and non-ASCII text, so the merges exercise every branch of the BPE loop.  The learner is
plain BPE training: count adjacent symbol pairs over the word frequencies, merge the most frequent
(ties: the lexicographically smallest pair), repeat.

Writes tests/golden/bpe_small_merges.txt.gz (data, committed).
"""
from __future__ import annotations

import collections
import gzip
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))

from federated_multi_modal_amd import tokenizer as T  # noqa: E402

N_MERGES = 1800

CLASSNAMES = """
airplane baseball_field basketball_court beach bridge cemetery chaparral christmas_tree_farm closed_road
coastal_mansion crosswalk dense_residential ferry_terminal football_field forest freeway golf_course harbor
intersection mobile_home_park nursing_home oil_gas_field oil_well overpass parking_lot parking_space railway
river runway runway_marking shipping_yard solar_panel sparse_residential storage_tank swimming_pool
tennis_court transformer_station wastewater_treatment_plant agricultural baseballdiamond buildings
denseresidential golfcourse mediumresidential mobilehomepark parkinglot sparseresidential storagetanks
tenniscourt annual_crop_land herbaceous_vegetation_land highway_or_road industrial_buildings pasture_land
permanent_crop_land residential_buildings sea_or_lake
"""

CAPTIONS = """
a photo of a dense residential area with many houses and trees.
an aerial view of a parking lot full of cars next to a large building.
a satellite image of a river running through green farmland near a small town.
there's a harbor with boats docked along the pier, and the water is calm.
the airport's runway has two airplanes waiting; it's a busy day.
a golf course with sand traps, ponds and a club house in the 18th hole.
a highway interchange with 4 lanes in each direction and an overpass.
storage tanks at an oil refinery, 12 of them in two rows.
we've seen solar panels covering the roof of the industrial buildings.
they'll build a new bridge over the lake by 2025; I'm sure they'd like to finish early.
a tennis court, a basketball court and a football field at the school.
sparse residential houses with swimming pools & large gardens.
the beach is crowded in summer: umbrellas, towels, people swimming.
crosswalks at the intersection of two roads in the city center.
a christmas tree farm with rows of small pine trees on a hill.
wastewater treatment plant with round basins (clarifiers) and pipes.
a cemetery with graves arranged in neat rows, surrounded by a wall.
annual crop land, permanent crop land and pasture land seen from above.
herbaceous vegetation land near a forest and a highway or road.
café in the plaza; the résumé of the naïve coöperative; jalapeño, über, façade.
東京 北京 ソウル 서울 москва αθήνα — emoji 🙂🛰️ and symbols © ® ™ ° ± × ÷.
numbers 0 1 2 3 4 5 6 7 8 9 10 100 2024 3.14 50% #1 @home $5 a-b a_b a/b.
"""


def corpus_words():
    freq = collections.Counter()
    text = CLASSNAMES.replace("_", " ") + "\n" + CAPTIONS * 3
    for line in text.split("\n"):
        for piece in T._SPLIT.findall(T.clean(line)):
            enc = T.byte_alphabet()
            freq["".join(enc[b] for b in piece.encode("utf-8"))] += 1
    return freq


def learn(freq, n_merges):
    words = {w: tuple(w[:-1]) + (w[-1] + "</w>",) for w in freq}
    merges = []
    for _ in range(n_merges):
        pairs = collections.Counter()
        for w, syms in words.items():
            for a, b in zip(syms, syms[1:]):
                pairs[(a, b)] += freq[w]
        if not pairs:
            break
        top = max(pairs.values())
        a, b = min(p for p, c in pairs.items() if c == top)
        merges.append((a, b))
        for w, syms in words.items():
            out, i = [], 0
            while i < len(syms):
                if i + 1 < len(syms) and syms[i] == a and syms[i + 1] == b:
                    out.append(a + b)
                    i += 2
                else:
                    out.append(syms[i])
                    i += 1
            words[w] = tuple(out)
    return merges


def main():
    merges = learn(corpus_words(), N_MERGES)
    body = "#version: 0.2 - synthetic merges (tests/golden/make_bpe_merges.py)\n" + "\n".join(f"{a} {b}" for a, b in merges)
    path = HERE / "bpe_small_merges.txt.gz"
    with open(path, "wb") as raw, gzip.GzipFile(filename="", mode="wb", fileobj=raw, mtime=0) as f:
        f.write(body.encode("utf-8"))
    print(f"wrote {path.name}: {len(merges)} merges")


if __name__ == "__main__":
    main()
