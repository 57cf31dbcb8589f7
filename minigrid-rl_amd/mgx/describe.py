"""PlaygroundEnv.llm_description and LLMDescriptionWrapper (src/environment.py:152-195) over the
engine: the scene text the reference's generators assemble while they place things
(custom_env.py:332-2034: 'The scene contains:' ... 'Mission: '), rebuilt from the engine's scene
record (mgx_scene: the env's current episode regenerated on the device, objs in placement order),
and the wrapper's 4,096-token mission observation (description + mission text, lower-cased,
indexed into the 32-symbol vocab).

The reference uses this only in manual mode (`make_env(manual=True)`: one env, GUI / LLM
planning).  The record needs the inline reset mode (`MgxEngine(..., ring_depth=-1)`), which keeps
each episode's generation start state.
"""
import ctypes

import numpy as np

from . import _lib

COLOR_NAMES = ("blue", "green", "grey", "purple", "red", "yellow")   # sorted(COLORS): objs colour index
TYPE_NAMES = {4: "door", 5: "key", 6: "ball", 7: "box", 8: "goal", 11: "door"}
T_DOOR, T_KEY, T_BOX, T_GOAL = 4, 5, 7, 8
SCENE_WORDS = 104               # MGX_SCENE_WORDS (include/mgx.h)
KEYFLAG = 1 << 24
MSN_LEN = 4096                  # LLMDescriptionWrapper.msn_len (environment.py:156)
VOCAB = [" ", "\n", "-", ":", ",", "."] + [chr(c) for c in range(ord("a"), ord("z") + 1)]   # environment.py:158-165

# multi-room layouts (custom_env.py:617-2034): layout line, door lines in door order, room names
_LAYOUT = {
    2: ("Two rooms. Left and right.\n", ["between the rooms\n"], ["Left", "Right"]),
    3: ("Three rooms. Upper left, lower left and right.\n",
        ["between the upper left and lower left rooms.\n", "between the upper left and right rooms.\n",
         "between the lower left and right rooms.\n"],
        ["Upper left", "Lower left", "Right"]),
    4: ("Four rooms. Upper left, lower left, upper right and lower right.\n",
        ["between the upper left and lower left rooms.\n", "between the upper right and lower right rooms.\n",
         "between the upper left and upper right rooms.\n", "between the lower left and lower right rooms.\n"],
        ["Upper left", "Lower left", "Upper right", "Lower right"]),
}


def _room_of(nr, x, y, mid):
    left, up = x < mid, y < mid
    if nr == 2:
        return 0 if left else 1
    if nr == 3:
        return (0 if up else 1) if left else 2
    return (0 if up else 1) if left else (2 if up else 3)


def scene(engine, env):
    """The scene record of env `env`'s current episode (include/mgx.h: mgx_scene) as a dict."""
    rec = (ctypes.c_uint32 * SCENE_WORDS)()
    _lib.check(engine.L.mgx_scene(engine.h, int(env), rec, engine._stream()), "mgx_scene")
    r = np.frombuffer(rec, dtype=np.uint32).copy()
    S = engine.size
    n = int(r[0])
    objs = []
    for w in r[8:8 + n]:
        w = int(w)
        objs.append(dict(type=w & 15, color=(w >> 4) & 15, x=(w >> 8) & 0xFF, y=(w >> 16) & 0xFF,
                         key=bool(w & KEYFLAG)))
    grid = r[8 + 32:].view(np.uint8)[:S * S].reshape(S, S)          # [y][x] cell codes
    return dict(objs=objs, agent=(int(r[1]) & 0xFF, (int(r[1]) >> 8) & 0xFF, (int(r[1]) >> 16) & 0xFF),
                mission_id=int(r[2]) & 0xFF, livelocks=int(r[3]), err=int(r[4]), grid=grid, size=S)


def _line(o):
    return "- goal\n" if o["type"] == T_GOAL else "- %s %s\n" % (COLOR_NAMES[o["color"]], TYPE_NAMES[o["type"]])


def llm_description(sc, problem):
    """PlaygroundEnv.llm_description for a scene record (custom_env.py: the generators' text)."""
    text = "The scene contains:\n"
    objs = sc["objs"]
    if problem != "multi":
        # single room (custom_env.py:332-593): every placed object in placement order, and the goal
        # -- except in _generate_drop_map, which places a goal but never mentions it (:543-545)
        text += "Only one room.\n"
        for o in objs:
            if not (o["type"] == T_GOAL and problem == "drp"):
                text += _line(o)
        return text + "Mission: "
    doors = [o for o in objs if o["type"] == T_DOOR and not o["key"]]
    nr = {1: 2, 3: 3, 4: 4}[len(doors)]
    S = sc["size"]
    mid = S // 2
    head, door_txt, rooms = _LAYOUT[nr]
    text += head
    for d, o in zip(door_txt, doors):
        locked = (int(sc["grid"][o["y"], o["x"]]) >> 7) & 1 and (int(sc["grid"][o["y"], o["x"]]) & 15) == T_DOOR
        text += "There is %s %s door %s" % ("a locked" if locked else "an unlocked", COLOR_NAMES[o["color"]], d)
    ax, ay, _ = sc["agent"]
    goal = [o for o in objs if o["type"] == T_GOAL][0]
    placed = [o for o in objs if o["type"] not in (T_DOOR, T_GOAL)]     # multi rooms hold no door objects
    for r, name in enumerate(rooms):
        # per room (e.g. custom_env.py:670-725): robot, the door keys placed here, goal, objects
        text += "%s room contains:\n" % name
        if _room_of(nr, ax, ay, mid) == r:
            text += "- robot\n"
        inside = [o for o in placed if _room_of(nr, o["x"], o["y"], mid) == r]
        for o in inside:
            if o["key"]:
                text += _line(o)
        if _room_of(nr, goal["x"], goal["y"], mid) == r:
            text += "- goal\n"
        for o in inside:
            if not o["key"]:
                text += _line(o)
    return text + "Mission: "


def mission_tokens(text):
    """LLMDescriptionWrapper._calculate_indexes (environment.py:170-179): int64 [4096]."""
    out = np.zeros(MSN_LEN, dtype=np.int64)
    for i, ch in enumerate(text.lower()):
        out[i] = VOCAB.index(ch)          # ValueError on a character outside the vocab, as the reference
    return out


class LLMDescriptionWrapper:
    """LLMDescriptionWrapper over an MgxEngine: observation(obs, env) replaces the mission tokens
    with the 4,096 indices of llm_description + mission text (environment.py:181-195)."""

    def __init__(self, engine, problem):
        if engine.ring_depth != 0:
            raise _lib.MgxError("LLMDescriptionWrapper needs MgxEngine(..., ring_depth=-1) (inline resets)")
        if not getattr(engine, "manual", False):
            # make_env(manual=True) is the only path that applies this wrapper (environment.py:19-20),
            # and its PlaygroundEnv ignores a premature 'done' (custom_env.py:325)
            raise _lib.MgxError("LLMDescriptionWrapper needs MgxEngine(..., manual=True) (make_env(manual=True))")
        self.engine, self.problem = engine, problem

    def description(self, env=0):
        return llm_description(scene(self.engine, env), self.problem)

    def observation(self, obs, env=0):
        sc = scene(self.engine, env)
        text = llm_description(sc, self.problem) + _lib.mission_text(sc["mission_id"])
        return {"direction": obs["direction"], "image": obs["image"], "mission": mission_tokens(text)}
