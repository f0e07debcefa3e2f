// Synthetic CloudFormation-shaped corpus (BASELINE.json configs[1]; SURVEY.md 8(d) cfg 2).
//
// Byte-identical to cloudformation-guard_amd/synth.py (`cfn_doc(i)` serialised with
// json.dumps(separators=(",", ":"))): doc i draws from xorshift32 seeded with 42 ^ i.  The
// generator lives natively so bench.py can stream 1M documents straight into the loader
// without a Python round trip; tests/test_synth_cpu.py pins the two generators together.
#include "synth_corpus.h"

#include <cstdio>
#include <cstdlib>

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

}  // namespace gg
