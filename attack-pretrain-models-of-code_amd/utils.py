"""Host-side attack utilities — the reference's `utils.py` interface, same names and behaviour.

Restates (reference file:line):
  GA operators           select_parents :84, mutate :92, crossover :99, map_chromesome :116
  identifier validity    is_valid_variable_{python,java,c} :126-148, is_valid_variable_name :150,
                         is_valid_substitue :162 (deny lists :13-78, incl. the missing-comma quirk
                         that fuses "getline" and "stdlib" into one entry)
  word handling          _tokenize :174, get_identifier_posistions_from_code :192,
                         get_masked_code_by_position :280
  MHM helpers            build_vocab :299, isUID :481, getUID :513
  datasets               CodeDataset :530
  misc                   set_seed :641, Recorder :651
The Python `random` call sequence of the GA operators is exactly the reference's, so a seeded run
draws the same mutants.  map_chromesome runs in the C++ host library (csrc/host/mutate.cpp).
"""
from __future__ import annotations

import csv
import os
import random
from keyword import iskeyword

import numpy as np

# --------------------------------------------------------------------------- deny lists (data)
JAVA_KEYWORDS = frozenset(
    "abstract assert boolean break byte case catch do double else enum extends final finally "
    "float for goto if implements import instanceof int interface long native new package "
    "private protected public return short static strictfp super switch throws transient try "
    "void volatile while".split())
JAVA_SPECIAL_IDS = frozenset(
    "main args Math System Random Byte Short Integer Long Float Double Character Boolean Data "
    "ParseException SimpleDateFormat Calendar Object String StringBuffer StringBuilder DateFormat "
    "Collection List Map Set Queue ArrayList HashSet HashMap".split())
C_KEYWORDS = frozenset(
    "auto break case char const continue default do double else enum extern float for goto if "
    "inline int long register restrict return short signed sizeof static struct switch typedef "
    "union unsigned void volatile while _Alignas _Alignof _Atomic _Bool _Complex _Generic "
    "_Imaginary _Noreturn _Static_assert _Thread_local __func__".split())
C_MACROS = frozenset(
    "NULL _IOFBF _IOLBF BUFSIZ EOF FOPEN_MAX TMP_MAX FILENAME_MAX L_tmpnam SEEK_CUR SEEK_END "
    "SEEK_SET EXIT_FAILURE EXIT_SUCCESS RAND_MAX MB_CUR_MAX".split())
# utils.py:39-78; note "getline" "stdlib" (missing comma) -> the single entry "getlinestdlib"
C_SPECIAL_IDS = frozenset(
    "main stdio cstdio stdio.h size_t FILE fpos_t stdin stdout stderr remove rename tmpfile tmpnam "
    "fclose fflush fopen freopen setbuf setvbuf fprintf fscanf printf scanf snprintf sprintf sscanf "
    "vprintf vscanf vsnprintf vsprintf vsscanf fgetc fgets fputc getc getchar putc putchar puts "
    "ungetc fread fwrite fgetpos fseek fsetpos ftell rewind clearerr feof ferror perror "
    "getlinestdlib cstdlib stdlib.h div_t ldiv_t lldiv_t atof atoi atol atoll strtod strtof "
    "strtold strtol strtoll strtoul strtoull rand srand aligned_alloc calloc malloc realloc free "
    "abort atexit exit at_quick_exit _Exit getenv quick_exit system bsearch qsort abs labs llabs "
    "div ldiv lldiv mblen mbtowc wctomb mbstowcs wcstombs string cstring string.h memcpy memmove "
    "memchr memcmp memset strcat strncat strchr strrchr strcmp strncmp strcoll strcpy strncpy "
    "strerror strlen strspn strcspn strpbrk strstr strtok strxfrm memccpy mempcpy strcat_s "
    "strcpy_s strdup strerror_r strlcat strlcpy strsignal strtok_r iostream istream ostream "
    "fstream sstream iomanip iosfwd ios wios streamoff streampos wstreampos streamsize cout cerr "
    "clog cin boolalpha noboolalpha skipws noskipws showbase noshowbase showpoint noshowpoint "
    "showpos noshowpos unitbuf nounitbuf uppercase nouppercase left right internal dec oct hex "
    "fixed scientific hexfloat defaultfloat width fill precision endl ends flush ws sin cos tan "
    "asin acos atan atan2 sinh cosh tanh exp sqrt log log10 pow powf ceil floor fabs cabs frexp "
    "ldexp modf fmod hypot poly matherr".split())
# MHM lists (utils.py:353-408): same keyword/macro/special sets plus the C operator list
MHM_OPS = frozenset(
    "... >>= <<= += -= *= /= %= &= ^= |= >> << ++ -- -> && || <= >= == != ; { <% } %> , : = ( ) "
    "[ <: ] :> . & ! ~ - + * / % < > ^ | ?".split())


# --------------------------------------------------------------------------- GA operators
# `rng` is the `random` module (the reference's global stream) or a `random.Random(seed)` of one
# attacked example (cross-example batching runs many examples' streams interleaved); both give the
# same draws for the same seed.
def select_parents(population, rng=random):
    """Two independent uniform picks (utils.py:84-90)."""
    idx = range(len(population))
    i1 = rng.choice(idx)
    i2 = rng.choice(idx)
    return population[i1], i1, population[i2], i2


def mutate(chromesome, variable_substitue_dict, rng=random):
    """In-place: one random gene gets a random substitute; returns the SAME dict (utils.py:92-97).
    Callers rely on the aliasing (attacker.py:228-238)."""
    pos = rng.choice(range(len(chromesome)))
    gene = list(chromesome.keys())[pos]
    chromesome[gene] = rng.choice(variable_substitue_dict[gene])
    return chromesome


def crossover(csome_1, csome_2, r=None, rng=random):
    """Single-point crossover at r (utils.py:99-113): child_1 takes csome_2's genes before r."""
    if r is None:
        r = rng.choice(range(len(csome_1)))
    child_1, child_2 = {}, {}
    for pos, name in enumerate(csome_1.keys()):
        first, second = (csome_2, csome_1) if pos < r else (csome_1, csome_2)
        child_1[name] = first[name]
        child_2[name] = second[name]
    return child_1, child_2


def map_chromesome(chromesome: dict, code: str, lang: str, example=None) -> str:
    """get_example_batch(code, chromesome, lang) (utils.py:116-120) via the C++ host library."""
    from .host import Example

    ex = example if example is not None else Example(code, lang)
    return ex.mutant_text(list(chromesome.items()))


# --------------------------------------------------------------------------- validity
def is_valid_variable_python(name: str) -> bool:
    return name.isidentifier() and not iskeyword(name)


def is_valid_variable_java(name: str) -> bool:
    return name.isidentifier() and name not in JAVA_KEYWORDS and name not in JAVA_SPECIAL_IDS


def is_valid_variable_c(name: str) -> bool:
    return (name.isidentifier() and name not in C_KEYWORDS and name not in C_MACROS
            and name not in C_SPECIAL_IDS)


def is_valid_variable_name(name: str, lang: str) -> bool:
    fn = {"python": is_valid_variable_python, "c": is_valid_variable_c,
          "java": is_valid_variable_java}.get(lang)
    return bool(fn and fn(name))


def is_valid_substitue(substitute: str, tgt_word: str, lang: str) -> bool:
    return is_valid_variable_name(substitute, lang)


# --------------------------------------------------------------------------- words
def _tokenize(seq, tokenizer):
    """utils.py:174-189: words = seq without '\\n' split on ' '; every word tokenised on its own
    (no leading-space marker).  Returns (words, sub_words(ids), keys)."""
    words = seq.replace("\n", "").split(" ")
    sub_words, keys, index = [], [], 0
    for word in words:
        sub = tokenizer.encode_ids(word) if hasattr(tokenizer, "encode_ids") else tokenizer.tokenize(word)
        sub_words += sub
        keys.append([index, index + len(sub)])
        index += len(sub)
    return words, sub_words, keys


def get_identifier_posistions_from_code(words_list: list, variable_names: list) -> dict:
    """utils.py:192-206: name -> word indices (names in the given order, only those present)."""
    positions = {}
    for name in variable_names:
        hits = [i for i, tok in enumerate(words_list) if tok == name]
        if hits:
            positions[name] = hits
    return positions


def get_masked_code_by_position(tokens: list, positions: dict):
    """utils.py:280-297: one copy per occurrence with that word replaced by '<unk>'."""
    masked, where = [], []
    for name in positions:
        for pos in positions[name]:
            masked.append(tokens[:pos] + ["<unk>"] + tokens[pos + 1:])
            where.append(pos)
    return masked, where


# --------------------------------------------------------------------------- MHM helpers
def build_vocab(codes, limit=5000):
    """utils.py:299-331: token counts with literal classes; returns (idx2txt, txt2idx)."""
    cnt = {"<str>": 0, "<char>": 0, "<int>": 0, "<fp>": 0}
    for c in codes:
        for t in c:
            if not t:
                continue
            if t[0] == '"' and t[-1] == '"':
                cnt["<str>"] += 1
            elif t[0] == "'" and t[-1] == "'":
                cnt["<char>"] += 1
            elif t[0] in "0123456789.":
                if "e" in t.lower():
                    cnt["<fp>"] += 1
                elif "." in t:
                    if t == ".":
                        cnt[t] = cnt.get(t, 0) + 1
                    else:
                        cnt["<fp>"] += 1
                else:
                    cnt["<int>"] += 1
            else:
                cnt[t] = cnt.get(t, 0) + 1
    ranked = sorted(cnt.items(), key=lambda kv: kv[1], reverse=True)
    idx2txt = ["<unk>", "<pad>"] + [k for i, (k, _) in enumerate(ranked) if i < limit - 1]
    return idx2txt, {t: i for i, t in enumerate(idx2txt)}


def isUID(_text=""):
    """utils.py:481-511 (note: only the inner characters [1:-1] are checked)."""
    t = _text.strip()
    if t == "" or " " in t or "\n" in t or "\r" in t:
        return False
    if t in C_KEYWORDS or t in MHM_OPS or t in C_MACROS or t in C_SPECIAL_IDS:
        return False
    if t[0].lower() in "0123456789" or "'" in t or '"' in t:
        return False
    if t[0].lower() not in "abcdefghijklmnopqrstuvwxyz_":
        return False
    return all(ch.lower() in "0123456789abcdefghijklmnopqrstuvwxyz_" for ch in t[1:-1])


def getUID(_tokens=(), uids=()):
    ids = {}
    for i, t in enumerate(_tokens):
        if isUID(t) and t in uids[0].keys():
            ids.setdefault(t, []).append(i)
    return ids


# --------------------------------------------------------------------------- datasets
class InputFeatures:
    """CodeXGLUE/Defect-detection/code/run.py:72-84."""

    def __init__(self, input_tokens, input_ids, idx, label):
        self.input_tokens = input_tokens
        self.input_ids = input_ids
        self.idx = str(idx)
        self.label = label


class CodeDataset:
    """utils.py:530-538 — items are (ids, label); ids as int64 tensors like the reference."""

    def __init__(self, examples):
        self.examples = examples

    def __len__(self):
        return len(self.examples)

    def __getitem__(self, i):
        import torch

        return torch.tensor(self.examples[i].input_ids), torch.tensor(self.examples[i].label)


class IdsDataset:
    """A pre-featurised batch: ids int32 [n, L] (+ lens) — what the engine consumes directly.
    len() is the query count the reference charges for the same batch."""

    def __init__(self, ids: np.ndarray, lens: np.ndarray | None = None, labels=None):
        self.ids = np.ascontiguousarray(ids, dtype=np.int32)
        self.lens = lens
        self.labels = labels

    def __len__(self):
        return self.ids.shape[0]

    def __getitem__(self, i):
        return self.ids[i], (self.labels[i] if self.labels is not None else 0)


def set_seed(seed=42):
    """utils.py:641-647 (the reference sets the misspelt PYHTONHASHSEED; kept)."""
    random.seed(seed)
    os.environ["PYHTONHASHSEED"] = str(seed)
    np.random.seed(seed)
    try:
        import torch

        torch.manual_seed(seed)
    except ImportError:
        pass


class Recorder:
    """utils.py:651-707: the attack result CSV (16 columns)."""

    HEADER = ["Index", "Original Code", "Program Length", "Adversarial Code", "True Label",
              "Original Prediction", "Adv Prediction", "Is Success", "Extracted Names",
              "Importance Score", "No. Changed Names", "No. Changed Tokens", "Replaced Names",
              "Attack Type", "Query Times", "Time Cost"]

    def __init__(self, file_path: str) -> None:
        self.file_path = file_path
        self.f = open(file_path, "w")
        self.writer = csv.writer(self.f)
        self.writer.writerow(self.HEADER)
        self.f.flush()  # a rank that writes no row still leaves a readable shard

    def close(self) -> None:
        if not self.f.closed:
            self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def write(self, index, code, prog_length, adv_code, true_label, orig_label, temp_label,
              is_success, variable_names, score_info, nb_changed_var, nb_changed_pos,
              replace_info, attack_type, query_times, time_cost):
        self.writer.writerow([index, code, prog_length, adv_code, true_label, orig_label,
                              temp_label, is_success, ",".join(variable_names), score_info,
                              nb_changed_var, nb_changed_pos, replace_info, attack_type,
                              query_times, time_cost])
        self.f.flush()

    def writemhm(self, index, code, prog_length, adv_code, true_label, orig_label, temp_label,
                 is_success, variable_names, score_info, nb_changed_var, nb_changed_pos,
                 replace_info, attack_type, query_times, time_cost):
        self.writer.writerow([index, code, prog_length, adv_code, true_label, orig_label,
                              temp_label, is_success, variable_names, score_info, nb_changed_var,
                              nb_changed_pos, replace_info, attack_type, query_times, time_cost])
        self.f.flush()
