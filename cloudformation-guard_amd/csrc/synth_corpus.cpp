// Synthetic CloudFormation-shaped corpus (BASELINE.json configs[1]; SURVEY.md 8(d) cfg 2).
//
// Byte-identical to cloudformation-guard_amd/synth.py (`cfn_doc(i)` serialised with
// json.dumps(separators=(",", ":"))): doc i draws from xorshift32 seeded with 42 ^ i.  The
// generator lives natively so bench.py can stream 1M documents straight into the loader
// without a Python round trip; tests/test_synth_cpu.py pins the two generators together.
#include "synth_corpus.h"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace gg {

namespace {

struct XorShift32 {
  uint32_t s;
  explicit XorShift32(uint32_t seed) : s(seed ? seed : 0x9E3779B9u) {}
  uint32_t next() {
    uint32_t x = s;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    s = x;
    return x;
  }
  bool chance(uint32_t per_mille) { return next() % 1000u < per_mille; }
  template <size_t N>
  const char* pick(const char* const (&v)[N]) { return v[next() % N]; }
  template <size_t N>
  int pick(const int (&v)[N]) { return v[next() % N]; }
};

const char* const kTypes[] = {"AWS::S3::Bucket", "AWS::IAM::Role", "AWS::EC2::Volume", "AWS::DynamoDB::Table",
                              "AWS::EC2::SecurityGroup", "AWS::Lambda::Function"};
const char* const kShort[] = {"Bucket", "Role", "Volume", "Table", "SecurityGroup", "Function"};

struct Out {
  std::string& s;
  void raw(const char* t) { s += t; }
  void str(const std::string& t) { s += '"'; s += t; s += '"'; }
  void key(const char* k) { s += '"'; s += k; s += "\":"; }
  void num(long long v) { s += std::to_string(v); }
  void boolean(bool b) { s += b ? "true" : "false"; }
};

std::string fmt(const char* f, long long a) {
  char buf[64];
  snprintf(buf, sizeof buf, f, a);
  return buf;
}

void resource(XorShift32& r, int t, int i, Out& o) {
  o.raw("{\"Type\":");
  o.str(kTypes[t]);
  o.raw(",\"Properties\":{");
  switch (t) {
    case 0: {  // AWS::S3::Bucket
      uint32_t suffix = r.next() % 100000u;
      o.key("BucketName");
      o.str("bucket-" + std::to_string(i) + "-" + std::to_string(suffix));
      if (r.chance(800)) {
        static const char* const alg[] = {"aws:kms", "AES256", "none"};
        o.raw(",\"BucketEncryption\":{\"ServerSideEncryptionConfiguration\":[{\"ServerSideEncryptionByDefault\":{\"SSEAlgorithm\":");
        o.str(r.pick(alg));
        o.raw("}}]}");
      }
      if (r.chance(800)) {
        o.raw(",\"LoggingConfiguration\":{\"DestinationBucketName\":");
        o.str(fmt("logs-%lld", i));
        o.raw("}");
      }
      if (r.chance(800)) {
        static const char* const keys[] = {"BlockPublicAcls", "BlockPublicPolicy", "IgnorePublicAcls", "RestrictPublicBuckets"};
        o.raw(",\"PublicAccessBlockConfiguration\":{");
        for (int k = 0; k < 4; k++) {
          if (k) o.raw(",");
          o.key(keys[k]);
          o.boolean(r.chance(900));
        }
        o.raw("}");
      }
      if (r.chance(800)) {
        static const char* const st[] = {"Enabled", "Suspended"};
        o.raw(",\"VersioningConfiguration\":{\"Status\":");
        o.str(r.pick(st));
        o.raw("}");
      }
      break;
    }
    case 1: {  // AWS::IAM::Role
      static const char* const svc[] = {"ec2.amazonaws.com", "lambda.amazonaws.com"};
      o.key("RoleName");
      o.str(fmt("role-%lld", i));
      o.raw(",\"AssumeRolePolicyDocument\":{\"Version\":\"2012-10-17\",\"Statement\":[{\"Effect\":\"Allow\",\"Principal\":{\"Service\":[");
      o.str(r.pick(svc));
      o.raw("]},\"Action\":[\"sts:AssumeRole\"]}]}");
      if (r.chance(800)) {
        static const char* const eff[] = {"Allow", "Deny"};
        static const char* const act[] = {"s3:*", "s3:GetObject", "*"};
        static const char* const res[] = {"*", "arn:aws:s3:::b/*"};
        o.raw(",\"Policies\":[{\"PolicyName\":");
        o.str(fmt("p%lld", i));
        o.raw(",\"PolicyDocument\":{\"Statement\":[{\"Effect\":");
        o.str(r.pick(eff));
        o.raw(",\"Action\":");
        o.str(r.pick(act));
        o.raw(",\"Resource\":");
        o.str(r.pick(res));
        o.raw("}]}}]");
      }
      break;
    }
    case 2: {  // AWS::EC2::Volume
      static const char* const az[] = {"us-east-1a", "us-west-2b"};
      o.key("Size");
      o.num(8 + r.next() % 500u);
      o.raw(",\"AvailabilityZone\":");
      o.str(r.pick(az));
      if (r.chance(800)) {
        o.raw(",\"Encrypted\":");
        o.boolean(r.chance(700));
      }
      break;
    }
    case 3: {  // AWS::DynamoDB::Table
      o.key("TableName");
      o.str(fmt("t%lld", i));
      o.raw(",\"KeySchema\":[{\"AttributeName\":\"id\",\"KeyType\":\"HASH\"}]");
      if (r.chance(800)) {
        o.raw(",\"SSESpecification\":{\"SSEEnabled\":");
        o.boolean(r.chance(800));
        o.raw("}");
      }
      break;
    }
    case 4: {  // AWS::EC2::SecurityGroup
      o.key("GroupDescription");
      o.str(fmt("sg %lld", i));
      if (r.chance(800)) {
        static const int ports[] = {22, 80, 443};
        static const char* const cidr[] = {"0.0.0.0/0", "10.0.0.0/8"};
        o.raw(",\"SecurityGroupIngress\":[{\"IpProtocol\":\"tcp\",\"FromPort\":");
        o.num(r.pick(ports));
        o.raw(",\"ToPort\":");
        o.num(r.pick(ports));
        o.raw(",\"CidrIp\":");
        o.str(r.pick(cidr));
        o.raw("}]");
      }
      break;
    }
    default: {  // AWS::Lambda::Function
      static const char* const rt[] = {"python3.9", "nodejs18.x"};
      static const char* const team[] = {"a", "b"};
      o.key("Runtime");
      o.str(r.pick(rt));
      o.raw(",\"Handler\":\"index.handler\"");
      if (r.chance(800)) {
        o.raw(",\"Tags\":[{\"Key\":\"team\",\"Value\":");
        o.str(r.pick(team));
        o.raw("}]");
      }
      break;
    }
  }
  o.raw("}");
  if (r.chance(100)) o.raw(",\"Metadata\":{\"guard\":{\"SuppressedRules\":[\"S3_BUCKET_LOGGING_ENABLED\"]}}");
  o.raw("}");
}

}  // namespace

void cfn_synth_doc(uint64_t index, int n_resources, std::string& s) {
  s.clear();
  // Diagnostic corpus shapes (A/B of lane divergence only; never set by bench.py or the tests):
  // GG_SYNTH_MOD=k generates doc (index % k); GG_SYNTH_SHAPE_GROUP=g gives the g consecutive docs
  // of a group one resource-type sequence (their property values still differ).
  static const uint64_t mod = getenv("GG_SYNTH_MOD") ? strtoull(getenv("GG_SYNTH_MOD"), nullptr, 10) : 0;
  static const uint64_t grp = getenv("GG_SYNTH_SHAPE_GROUP") ? strtoull(getenv("GG_SYNTH_SHAPE_GROUP"), nullptr, 10) : 0;
  if (mod) index %= mod;
  XorShift32 r((uint32_t)(42u ^ (uint32_t)index));
  XorShift32 rt((uint32_t)(0x5eedu ^ (uint32_t)(grp ? index / grp : 0)));
  Out o{s};
  o.raw("{\"AWSTemplateFormatVersion\":\"2010-09-09\",\"Resources\":{");
  for (int k = 0; k < n_resources; k++) {
    int t = (int)(r.next() % 6u);
    if (grp) t = (int)(rt.next() % 6u);
    if (k) o.raw(",");
    s += "\"Res" + std::to_string(k) + kShort[t] + "\":";
    resource(r, t, k, o);
  }
  o.raw("}}");
}

// ---- block-style YAML (synth.py cfn_yaml_doc, byte-identical; tests/test_synth_cpu.py) ------------------
namespace {

// the generator's JSON as a tree (its own compact output: strings without escapes, ints, bools)
struct YV {
  int kind = 0;   // 0 string, 1 int, 2 bool, 3 map, 4 list
  std::string s;
  long long i = 0;
  bool b = false;
  std::vector<std::pair<std::string, YV>> m;
  std::vector<YV> a;
};

struct JP {
  const std::string& t;
  size_t p = 0;
  std::string str() {
    std::string r;
    p++;
    while (t[p] != '"') r += t[p++];
    p++;
    return r;
  }
  YV val() {
    YV v;
    const char c = t[p];
    if (c == '"') { v.kind = 0; v.s = str(); }
    else if (c == '{') {
      v.kind = 3; p++;
      while (t[p] != '}') { std::string k = str(); p++; YV x = val(); v.m.emplace_back(std::move(k), std::move(x)); if (t[p] == ',') p++; }
      p++;
    } else if (c == '[') {
      v.kind = 4; p++;
      while (t[p] != ']') { v.a.push_back(val()); if (t[p] == ',') p++; }
      p++;
    } else if (c == 't' || c == 'f') { v.kind = 2; v.b = c == 't'; p += v.b ? 4 : 5; }
    else { v.kind = 1; size_t e = p; while (t[e] == '-' || (t[e] >= '0' && t[e] <= '9')) e++; v.i = std::stoll(t.substr(p, e - p)); p = e; }
    return v;
  }
};

bool numeric_like(const std::string& s) {
  std::string t = (!s.empty() && (s[0] == '+' || s[0] == '-')) ? s.substr(1) : s;
  std::string low;
  for (char c : t) low += (char)tolower((unsigned char)c);
  if (low == "inf" || low == "infinity" || low == "nan") return true;
  bool digits = false, all = true;
  for (char c : t) {
    if (c >= '0' && c <= '9') digits = true;
    else if (!(c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-')) all = false;
  }
  return digits && all;
}

bool plain_ok(const std::string& s, bool flow = false) {
  static const char* const words[] = {"true", "false", "yes", "no", "on", "off", "y", "n", "~", "null", "Null", "NULL", "True",
                                      "False", "TRUE", "FALSE", "Yes", "No", "YES", "NO", "On", "Off", "ON", "OFF", "Y", "N"};
  if (s.empty() || s.front() == ' ' || s.back() == ' ' || s.front() == '\n' || s.back() == '\n') return false;
  for (const char* w : words) if (s == w) return false;
  if (numeric_like(s)) return false;
  if (std::string("-?:,[]{}#&*!|>'\"%@`").find(s[0]) != std::string::npos) return false;
  if (s.find(": ") != std::string::npos || s.find(" #") != std::string::npos || s.back() == ':' || s.find('\n') != std::string::npos) return false;
  for (unsigned char c : s) if (c < 0x20 || c >= 0x7F) return false;
  if (flow) for (char c : s) if (std::string(",[]{}:").find(c) != std::string::npos) return false;
  return true;
}

std::string jdump(const std::string& s) {
  std::string r = "\"";
  for (char c : s) { if (c == '"' || c == '\\') r += '\\'; r += c; }
  return r + "\"";
}

std::string yscalar(const YV& v, XorShift32& r, bool flow = false) {
  if (v.kind == 2) return v.b ? "true" : "false";
  if (v.kind == 1) return std::to_string(v.i);
  const uint32_t pick = r.next() % 5u;
  if (plain_ok(v.s, flow) && pick < 3) return v.s;
  bool simple = v.s.find('\\') == std::string::npos;
  for (unsigned char c : v.s) if (c < 0x20 || c >= 0x7F) simple = false;
  if (pick == 3 && simple) {
    std::string q = "'";
    for (char c : v.s) { q += c; if (c == '\'') q += '\''; }
    return q + "'";
  }
  return jdump(v.s);
}

std::string ykey(const std::string& k, XorShift32& r) { return (plain_ok(k) && r.next() % 6u) ? k : jdump(k); }

std::string lower(const std::string& s) {
  std::string r;
  for (char c : s) r += (char)tolower((unsigned char)c);
  return r;
}

void ylines(const YV& v, int indent, XorShift32& r, std::vector<std::string>& out) {
  const std::string pad(indent, ' ');
  if (v.kind == 3) {
    for (auto& kv : v.m) {
      const YV& x = kv.second;
      if (r.next() % 13u == 0) out.push_back(pad + "# " + lower(kv.first));
      const std::string key = ykey(kv.first, r);
      if (x.kind == 3 && !x.m.empty()) {
        out.push_back(pad + key + ":");
        ylines(x, indent + 2, r, out);
      } else if (x.kind == 4 && !x.a.empty()) {
        bool scalars = true;
        for (auto& e : x.a) if (e.kind >= 3) scalars = false;
        bool flow = false;
        if (scalars && r.next() % 3u == 0) {
          flow = true;
          for (auto& e : x.a) if (e.kind == 0 && !plain_ok(e.s, true)) flow = false;
        }
        if (flow) {
          std::string f;
          for (size_t j = 0; j < x.a.size(); j++) { if (j) f += ", "; f += yscalar(x.a[j], r, true); }
          out.push_back(pad + key + ": [" + f + "]");
        } else {
          out.push_back(pad + key + ":");
          ylines(x, indent + (r.next() % 2u ? 2 : 0), r, out);
        }
      } else if (x.kind == 3) {
        out.push_back(pad + key + ": {}");
      } else if (x.kind == 4) {
        out.push_back(pad + key + ": []");
      } else {
        const std::string tail = r.next() % 17u == 0 ? "  # note" : "";
        out.push_back(pad + key + ": " + yscalar(x, r) + tail);
      }
    }
  } else {
    for (auto& x : v.a) {
      if (x.kind == 3 && !x.m.empty()) {
        std::vector<std::string> sub;
        ylines(x, indent + 2, r, sub);
        out.push_back(pad + "- " + sub[0].substr(indent + 2));
        for (size_t j = 1; j < sub.size(); j++) out.push_back(sub[j]);
      } else if (x.kind == 4 && !x.a.empty()) {
        out.push_back(pad + "-");
        ylines(x, indent + 2, r, out);
      } else if (x.kind >= 3) {
        out.push_back(pad + "- " + (x.kind == 3 ? "{}" : "[]"));
      } else {
        out.push_back(pad + "- " + yscalar(x, r));
      }
    }
  }
}

}  // namespace

void cfn_synth_yaml_doc(uint64_t index, int n_resources, std::string& out) {
  std::string json;
  cfn_synth_doc(index, n_resources, json);
  JP jp{json};
  const YV root = jp.val();
  uint32_t seed = 0x9E3779B9u ^ (uint32_t)((index * 2654435761ull) & 0xFFFFFFFFull);
  if (!seed) seed = 1;
  XorShift32 r(seed);
  std::vector<std::string> lines;
  if (r.next() % 3u == 0) lines.push_back("---");
  if (r.next() % 2u) lines.push_back("# synthetic template " + std::to_string(index));
  ylines(root, 0, r, lines);
  out.clear();
  for (size_t j = 0; j < lines.size(); j++) { if (j) out += '\n'; out += lines[j]; }
  out += '\n';
}

}  // namespace gg
