"""Extract the bot-vs-bot outcomes of the reference's league database.

Reads /root/reference/experiments/gym-microrts-static-files/league.db (SQLite,
opened read-only through the stdlib -- a data file, nothing in it executes) and
writes tests/golden/league_outcomes.json: for every ordered pair (challenger =
player 0, defender = player 1) among the built-in bots the oracle and the
device restate, the summed (win, draw, loss) of the challenger.  The matches
were played by /root/reference/experiments/league.py:236-245, 324-338
(MicroRTSBotVecEnv, basesWorkers16x16A, max_steps 5000, WinLoss from player 0's
view; 5 matches per ordered pair).  Run here only (the reference is absent on
the GPU box); the JSON is the committed fixture.
"""
import json
import os
import sqlite3
from collections import defaultdict

DB = "/root/reference/experiments/gym-microrts-static-files/league.db"
BOTS = ["passiveAI", "randomBiasedAI", "randomAI", "lightRushAI", "workerRushAI", "coacAI"]


def main():
    con = sqlite3.connect(f"file:{DB}?mode=ro", uri=True)
    names = dict(con.execute("select id, name from ai").fetchall())
    agg = defaultdict(lambda: [0, 0, 0])
    for c, d, w, dr, l in con.execute("select challenger_id, defender_id, win, draw, loss from matchhistory"):
        a, b = names[c], names[d]
        if a in BOTS and b in BOTS:
            r = agg[(a, b)]
            r[0] += w
            r[1] += dr
            r[2] += l
    con.close()
    out = {
        "source": "experiments/gym-microrts-static-files/league.db (matchhistory), experiments/league.py:236-245",
        "map": "maps/16x16/basesWorkers16x16A.xml",
        "max_steps": 5000,
        "pairs": [{"p0": a, "p1": b, "win": v[0], "draw": v[1], "loss": v[2]} for (a, b), v in sorted(agg.items())],
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "league_outcomes.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(out['pairs'])} ordered pairs -> {path}")


if __name__ == "__main__":
    main()
