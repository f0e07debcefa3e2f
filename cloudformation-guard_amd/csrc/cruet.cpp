// Key case converters tried on a key miss (guard/src/rules/eval_context.rs:315-326, 539-568).
// cruet 0.14.0 (Cargo.lock) is not vendored in the reference; this restates its published
// algorithm (Inflector-style to_case_camel_like / to_case_snake_like).  The compiler precomputes
// the seven alternates of every query key so the device only compares hashes.
#include <regex>
#include <string>
#include <vector>

namespace gg {

namespace {

bool alnum_cp(unsigned char c) { return isalnum(c) || c >= 0x80; }

std::string trim_right(const std::string& s) {
  size_t i = s.size();
  while (i > 0 && !alnum_cp((unsigned char)s[i - 1])) i--;
  return s.substr(0, i);
}

char up(char c) { return (c >= 'a' && c <= 'z') ? (char)(c - 32) : c; }
char low(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c; }
bool is_upper(char c) { return c >= 'A' && c <= 'Z'; }
bool is_lower(char c) { return c >= 'a' && c <= 'z'; }
bool is_num(char c) { return c >= '0' && c <= '9'; }

std::string camel_like(const std::string& s, bool new_word, bool first_word, char inj, bool has_sep, bool inverted) {
  char last = ' ';
  bool found = false;
  std::string out;
  for (char ch : trim_right(s)) {
    bool an = alnum_cp((unsigned char)ch);
    if (!an && found) new_word = true;
    else if (!found && !an) continue;
    else if (is_num(ch)) { found = true; new_word = true; out.push_back(ch); }
    else if (new_word || (is_lower(last) && is_upper(ch) && last != ' ')) {
      found = true; new_word = false;
      if (has_sep && !first_word) out.push_back(inj);
      if (!inverted || first_word) out.push_back(up(ch)); else out.push_back(low(ch));
      first_word = false;
    } else { found = true; last = ch; out.push_back(low(ch)); }
  }
  return out;
}

std::string snake_like(const std::string& s, char sep) {
  bool first = true;
  std::string out;
  std::string t = trim_right(s);
  for (size_t idx = 0; idx < t.size(); idx++) {
    char ch = t[idx];
    if (!alnum_cp((unsigned char)ch)) {
      if (!first) { first = true; out.push_back(sep); }
      continue;
    }
    bool needs = false;
    if (!first && ch == up(ch)) {
      char nx = idx + 1 < s.size() ? s[idx + 1] : 'A';
      char pv = idx >= 1 && idx - 1 < s.size() ? s[idx - 1] : 'A';
      needs = is_lower(nx) || is_lower(pv);
    }
    first = false;
    if (needs) out.push_back(sep);
    out.push_back(low(ch));
  }
  return out;
}

const char* UNCOUNTABLE[] = {
    "accommodation", "adulthood", "advertising", "advice", "aggression", "aid", "air", "aircraft", "alcohol",
    "anger", "applause", "arithmetic", "assistance", "athletics", "bacon", "baggage", "beef", "biology", "blood",
    "botany", "bread", "butter", "carbon", "cardboard", "cash", "chalk", "chaos", "chess", "crossroads",
    "countryside", "dancing", "deer", "dignity", "dirt", "dust", "economics", "education", "electricity",
    "engineering", "enjoyment", "envy", "equipment", "ethics", "evidence", "evolution", "fame", "fiction", "flour",
    "flu", "food", "fuel", "fun", "furniture", "gallows", "garbage", "garlic", "genetics", "gold", "golf", "gossip",
    "grammar", "gratitude", "grief", "guilt", "gymnastics", "happiness", "hardware", "harm", "hate", "hatred",
    "health", "heat", "help", "homework", "honesty", "honey", "hospitality", "housework", "humour", "hunger",
    "hydrogen", "ice", "importance", "inflation", "information", "innocence", "iron", "irony", "jam", "jewelry",
    "judo", "karate", "knowledge", "lack", "laughter", "lava", "leather", "leisure", "lightning", "linguine",
    "linguini", "linguistics", "literature", "litter", "livestock", "logic", "loneliness", "luck", "luggage",
    "macaroni", "machinery", "magic", "management", "mankind", "marble", "mathematics", "mayonnaise", "measles",
    "methane", "milk", "money", "mud", "music", "mumps", "nature", "news", "nitrogen", "nonsense", "nurture",
    "nutrition", "obedience", "obesity", "oxygen", "pasta", "patience", "physics", "poetry", "pollution",
    "poverty", "pride", "psychology", "publicity", "punctuation", "quartz", "racism", "relaxation", "reliability",
    "research", "respect", "revenge", "rice", "rubbish", "rum", "safety", "scenery", "seafood", "seaside",
    "series", "shame", "sheep", "shopping", "sleep", "smoke", "smoking", "snow", "soap", "software", "soil",
    "spaghetti", "species", "steam", "stuff", "stupidity", "sunshine", "symmetry", "tennis", "thirst", "thunder",
    "timber", "traffic", "transportation", "trust", "underwear", "unemployment", "unity", "validity", "veal",
    "vegetation", "vegetarianism", "vengeance", "violence", "vitality", "warmth", "wealth", "weather", "welfare",
    "wheat", "wildlife", "wisdom", "yoga", "zinc", "zoology"};

const char* SPECIAL[][2] = {{"oxen", "ox"}, {"boxes", "box"}, {"men", "man"}, {"women", "woman"}, {"dice", "die"},
                            {"yes", "yes"}, {"feet", "foot"}, {"eaves", "eave"}, {"geese", "goose"},
                            {"teeth", "tooth"}, {"quizzes", "quiz"}};

const char* RULES[][2] = {
    {"(\\w*)s$", "$1"},
    {"(\\w*)(ss)$", "$1$2"},
    {"(n)ews$", "$1ews"},
    {"(\\w*)(o)es$", "$1$2"},
    {"(\\w*)([ti])a$", "$1$2um"},
    {"((a)naly|(b)a|(d)iagno|(p)arenthe|(p)rogno|(s)ynop|(t)he)(sis|ses)$", "$1sis"},
    {"(^analy)(sis|ses)$", "$1sis"},
    {"(\\w*)([^f])ves$", "$1$2fe"},
    {"(\\w*)(hive)s$", "$1$2"},
    {"(\\w*)(tive)s$", "$1$2"},
    {"(\\w*)([lr])ves$", "$1$2f"},
    {"(\\w*([^aeiouy]|qu))ies$", "$1y"},
    {"(s)eries$", "$1eries"},
    {"(m)ovies$", "$1ovie"},
    {"(\\w*)(x|ch|ss|sh)es$", "$1$2"},
    {"(m|l)ice$", "$1ouse"},
    {"(bus)(es)?$", "$1"},
    {"(shoe)s$", "$1"},
    {"(cris|ax|test)es$", "$1is"},
    {"(octop|vir)(us|i)$", "$1us"},
    {"(alias|status)(es)?$", "$1"},
    {"^(ox)en", "$1"},
    {"(vert|ind)ices$", "$1ex"},
    {"(matr)ices$", "$1ix"},
    {"(quiz)zes$", "$1"},
    {"(database)s$", "$1"},
};

std::string to_singular(const std::string& s) {
  for (const char* u : UNCOUNTABLE) if (s == u) return s;
  for (auto& sp : SPECIAL) if (s == sp[0]) return sp[1];
  static std::vector<std::regex> rx;
  if (rx.empty()) for (auto& r : RULES) rx.emplace_back(r[0]);
  for (int k = (int)(sizeof RULES / sizeof *RULES) - 1; k >= 0; k--) {
    if (std::regex_search(s, rx[k])) return std::regex_replace(s, rx[k], RULES[k][1], std::regex_constants::format_first_only);
  }
  return s;
}

}  // namespace

std::string to_camel_case(const std::string& s) { return camel_like(s, false, false, ' ', false, false); }
std::string to_pascal_case(const std::string& s) { return camel_like(s, true, false, ' ', false, false); }
std::string to_title_case(const std::string& s) { return camel_like(s, true, true, ' ', true, false); }
std::string to_train_case(const std::string& s) { return camel_like(s, true, true, '-', true, false); }
std::string to_snake_case(const std::string& s) { return snake_like(s, '_'); }
std::string to_kebab_case(const std::string& s) { return snake_like(s, '-'); }
std::string to_class_case(const std::string& s) {
  std::string plural = to_pascal_case(s);
  size_t pos = 0;
  for (size_t i = plural.size(); i-- > 0;) if (is_upper(plural[i])) { pos = i; break; }
  return plural.substr(0, pos) + to_singular(plural.substr(pos));
}

// CONVERTERS order: camel, class, kebab, pascal, snake, title, train
void key_alternates(const std::string& key, std::string out[7]) {
  out[0] = to_camel_case(key);
  out[1] = to_class_case(key);
  out[2] = to_kebab_case(key);
  out[3] = to_pascal_case(key);
  out[4] = to_snake_case(key);
  out[5] = to_title_case(key);
  out[6] = to_train_case(key);
}

}  // namespace gg
