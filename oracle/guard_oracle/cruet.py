"""Key case converters (TEST INFRASTRUCTURE ONLY -- the parity oracle).

The reference tries, on a key miss, the seven cruet 0.14.0 case converters in the order of
``CONVERTERS`` (``guard/src/rules/eval_context.rs:315-326``).  cruet is a third-party crate
(a fork of Inflector 0.11) and is not vendored under /root/reference, so this restates its
published algorithm (``to_case_camel_like`` / ``to_case_snake_like``).  The class-case
converter singularizes the last word; the singular rule table below is the Rails/Inflector
English table, pinned only by the reference's own converter test
(``eval_context_tests.rs:409-456``) -- beyond that it is "parity unpinned".
"""
import re


def _is_alnum(c):
    return c.isalnum()


def _trim_right(s):
    i = len(s)
    while i > 0 and not _is_alnum(s[i - 1]):
        i -= 1
    return s[:i]


def _ascii_upper(c):
    return c.upper() if "a" <= c <= "z" else c


def _ascii_lower(c):
    return c.lower() if "A" <= c <= "Z" else c


def _camel_like(s, new_word, first_word, injectable, has_sep, inverted):
    last_char = " "
    found_real = False
    out = []
    for ch in _trim_right(s):
        if (not _is_alnum(ch)) and found_real:
            new_word = True
        elif (not found_real) and not _is_alnum(ch):
            continue
        elif ch.isnumeric():
            found_real = True
            new_word = True
            out.append(ch)
        elif new_word or (last_char.islower() and ch.isupper() and last_char != " "):
            found_real = True
            new_word = False
            if has_sep and not first_word:
                out.append(injectable)
            if (not inverted) or first_word:
                out.append(_ascii_upper(ch))
            else:
                out.append(_ascii_lower(ch))
            first_word = False
        else:
            found_real = True
            last_char = ch
            out.append(_ascii_lower(ch))
    return "".join(out)


def _snake_like(s, sep, upper=False):
    first = True
    out = []
    chars = list(s)
    conv = _ascii_upper if upper else _ascii_lower
    # char_indices() yields byte offsets; the reference then indexes chars().nth() with them
    t = _trim_right(s)
    byte_off = 0
    for ch in t:
        idx = byte_off
        byte_off += len(ch.encode("utf-8"))
        if not _is_alnum(ch):
            if not first:
                first = True
                out.append(sep)
        elif (not first) and ch == _ascii_upper(ch) and _neighbour_lower(chars, idx):
            first = False
            out.append(sep)
            out.append(conv(ch))
        else:
            first = False
            out.append(conv(ch))
    return "".join(out)


def _neighbour_lower(chars, idx):
    nxt = chars[idx + 1] if idx + 1 < len(chars) else "A"
    prv = chars[idx - 1] if 0 <= idx - 1 < len(chars) else "A"
    return nxt.islower() or prv.islower()


def to_camel_case(s):
    return _camel_like(s, False, False, " ", False, False)


def to_pascal_case(s):
    return _camel_like(s, True, False, " ", False, False)


def to_title_case(s):
    return _camel_like(s, True, True, " ", True, False)


def to_train_case(s):
    return _camel_like(s, True, True, "-", True, False)


def to_snake_case(s):
    return _snake_like(s, "_")


def to_kebab_case(s):
    return _snake_like(s, "-")


UNCOUNTABLE = {
    "accommodation", "adulthood", "advertising", "advice", "aggression", "aid", "air", "aircraft",
    "alcohol", "anger", "applause", "arithmetic", "assistance", "athletics", "bacon", "baggage",
    "beef", "biology", "blood", "botany", "bread", "butter", "carbon", "cardboard", "cash", "chalk",
    "chaos", "chess", "crossroads", "countryside", "dancing", "deer", "dignity", "dirt", "dust",
    "economics", "education", "electricity", "engineering", "enjoyment", "envy", "equipment",
    "ethics", "evidence", "evolution", "fame", "fiction", "flour", "flu", "food", "fuel", "fun",
    "furniture", "gallows", "garbage", "garlic", "genetics", "gold", "golf", "gossip", "grammar",
    "gratitude", "grief", "guilt", "gymnastics", "happiness", "hardware", "harm", "hate", "hatred",
    "health", "heat", "help", "homework", "honesty", "honey", "hospitality", "housework", "humour",
    "hunger", "hydrogen", "ice", "importance", "inflation", "information", "innocence", "iron",
    "irony", "jam", "jewelry", "judo", "karate", "knowledge", "lack", "laughter", "lava", "leather",
    "leisure", "lightning", "linguine", "linguini", "linguistics", "literature", "litter",
    "livestock", "logic", "loneliness", "luck", "luggage", "macaroni", "machinery", "magic",
    "management", "mankind", "marble", "mathematics", "mayonnaise", "measles", "methane", "milk",
    "money", "mud", "music", "mumps", "nature", "news", "nitrogen", "nonsense", "nurture",
    "nutrition", "obedience", "obesity", "oxygen", "pasta", "patience", "physics", "poetry",
    "pollution", "poverty", "pride", "psychology", "publicity", "punctuation", "quartz", "racism",
    "relaxation", "reliability", "research", "respect", "revenge", "rice", "rubbish", "rum",
    "safety", "scenery", "seafood", "seaside", "series", "shame", "sheep", "shopping", "sleep",
    "smoke", "smoking", "snow", "soap", "software", "soil", "spaghetti", "species", "steam",
    "stuff", "stupidity", "sunshine", "symmetry", "tennis", "thirst", "thunder", "timber",
    "traffic", "transportation", "trust", "underwear", "unemployment", "unity", "validity",
    "veal", "vegetation", "vegetarianism", "vengeance", "violence", "vitality", "warmth",
    "wealth", "weather", "welfare", "wheat", "wildlife", "wisdom", "yoga", "zinc", "zoology",
}

_SPECIAL = {"oxen": "ox", "boxes": "box", "men": "man", "women": "woman", "dice": "die", "yes": "yes",
            "feet": "foot", "eaves": "eave", "geese": "goose", "teeth": "tooth", "quizzes": "quiz"}

# (pattern, replacement) -- applied last-to-first, first match wins
_RULES = [
    (r"(\w*)s$", r"\1"),
    (r"(\w*)(ss)$", r"\1\2"),
    (r"(n)ews$", r"\1ews"),
    (r"(\w*)(o)es$", r"\1\2"),
    (r"(\w*)([ti])a$", r"\1\2um"),
    (r"((a)naly|(b)a|(d)iagno|(p)arenthe|(p)rogno|(s)ynop|(t)he)(sis|ses)$", r"\1sis"),
    (r"(^analy)(sis|ses)$", r"\1sis"),
    (r"(\w*)([^f])ves$", r"\1\2fe"),
    (r"(\w*)(hive)s$", r"\1\2"),
    (r"(\w*)(tive)s$", r"\1\2"),
    (r"(\w*)([lr])ves$", r"\1\2f"),
    (r"(\w*([^aeiouy]|qu))ies$", r"\1y"),
    (r"(s)eries$", r"\1eries"),
    (r"(m)ovies$", r"\1ovie"),
    (r"(\w*)(x|ch|ss|sh)es$", r"\1\2"),
    (r"(m|l)ice$", r"\1ouse"),
    (r"(bus)(es)?$", r"\1"),
    (r"(shoe)s$", r"\1"),
    (r"(cris|ax|test)es$", r"\1is"),
    (r"(octop|vir)(us|i)$", r"\1us"),
    (r"(alias|status)(es)?$", r"\1"),
    (r"^(ox)en", r"\1"),
    (r"(vert|ind)ices$", r"\1ex"),
    (r"(matr)ices$", r"\1ix"),
    (r"(quiz)zes$", r"\1"),
    (r"(database)s$", r"\1"),
]
_RULES_C = [(re.compile(p), r) for p, r in _RULES]


def to_singular(s):
    if s in UNCOUNTABLE:
        return s
    if s in _SPECIAL:
        return _SPECIAL[s]
    for rx, rep in reversed(_RULES_C):
        if rx.search(s):
            return rx.sub(rep, s, count=1)
    return s


def to_class_case(s):
    plural = to_pascal_case(s)
    pos = 0
    for i in range(len(plural) - 1, -1, -1):
        if plural[i].isupper():
            pos = i
            break
    return plural[:pos] + to_singular(plural[pos:])


CONVERTERS = [to_camel_case, to_class_case, to_kebab_case, to_pascal_case, to_snake_case,
              to_title_case, to_train_case]
