"""Synthetic CloudFormation-shaped corpora (BASELINE.json configs; SURVEY.md 8d cfg 2).

Doc i is generated from xorshift32 seeded with 42 ^ i: 50 resources drawn uniformly from six
types, each optional property present with probability ~0.8.  Output is compact JSON text.
"""
import json

TYPES = ["AWS::S3::Bucket", "AWS::IAM::Role", "AWS::EC2::Volume", "AWS::DynamoDB::Table",
         "AWS::EC2::SecurityGroup", "AWS::Lambda::Function"]


class XorShift32:
    def __init__(self, seed):
        self.s = (seed & 0xFFFFFFFF) or 0x9E3779B9

    def next(self):
        x = self.s
        x ^= (x << 13) & 0xFFFFFFFF
        x ^= x >> 17
        x ^= (x << 5) & 0xFFFFFFFF
        self.s = x & 0xFFFFFFFF
        return self.s

    def chance(self, p):
        return (self.next() % 1000) < int(p * 1000)

    def pick(self, seq):
        return seq[self.next() % len(seq)]


def _resource(r, t, i):
    props = {}
    if t == "AWS::S3::Bucket":
        props["BucketName"] = "bucket-%d-%d" % (i, r.next() % 100000)
        if r.chance(0.8):
            props["BucketEncryption"] = {"ServerSideEncryptionConfiguration": [
                {"ServerSideEncryptionByDefault": {"SSEAlgorithm": r.pick(["aws:kms", "AES256", "none"])}}]}
        if r.chance(0.8):
            props["LoggingConfiguration"] = {"DestinationBucketName": "logs-%d" % i}
        if r.chance(0.8):
            props["PublicAccessBlockConfiguration"] = {k: r.chance(0.9) for k in (
                "BlockPublicAcls", "BlockPublicPolicy", "IgnorePublicAcls", "RestrictPublicBuckets")}
        if r.chance(0.8):
            props["VersioningConfiguration"] = {"Status": r.pick(["Enabled", "Suspended"])}
    elif t == "AWS::IAM::Role":
        props["RoleName"] = "role-%d" % i
        props["AssumeRolePolicyDocument"] = {"Version": "2012-10-17", "Statement": [
            {"Effect": "Allow", "Principal": {"Service": [r.pick(["ec2.amazonaws.com", "lambda.amazonaws.com"])]},
             "Action": ["sts:AssumeRole"]}]}
        if r.chance(0.8):
            props["Policies"] = [{"PolicyName": "p%d" % i, "PolicyDocument": {"Statement": [
                {"Effect": r.pick(["Allow", "Deny"]), "Action": r.pick(["s3:*", "s3:GetObject", "*"]),
                 "Resource": r.pick(["*", "arn:aws:s3:::b/*"])}]}}]
    elif t == "AWS::EC2::Volume":
        props["Size"] = 8 + r.next() % 500
        props["AvailabilityZone"] = r.pick(["us-east-1a", "us-west-2b"])
        if r.chance(0.8):
            props["Encrypted"] = r.chance(0.7)
    elif t == "AWS::DynamoDB::Table":
        props["TableName"] = "t%d" % i
        props["KeySchema"] = [{"AttributeName": "id", "KeyType": "HASH"}]
        if r.chance(0.8):
            props["SSESpecification"] = {"SSEEnabled": r.chance(0.8)}
    elif t == "AWS::EC2::SecurityGroup":
        props["GroupDescription"] = "sg %d" % i
        if r.chance(0.8):
            props["SecurityGroupIngress"] = [{"IpProtocol": "tcp", "FromPort": r.pick([22, 80, 443]),
                                              "ToPort": r.pick([22, 80, 443]),
                                              "CidrIp": r.pick(["0.0.0.0/0", "10.0.0.0/8"])}]
    else:
        props["Runtime"] = r.pick(["python3.9", "nodejs18.x"])
        props["Handler"] = "index.handler"
        if r.chance(0.8):
            props["Tags"] = [{"Key": "team", "Value": r.pick(["a", "b"])}]
    res = {"Type": t, "Properties": props}
    if r.chance(0.1):
        res["Metadata"] = {"guard": {"SuppressedRules": ["S3_BUCKET_LOGGING_ENABLED"]}}
    return res


def cfn_doc(i, n_resources=50):
    r = XorShift32(42 ^ i)
    resources = {}
    for k in range(n_resources):
        t = TYPES[r.next() % len(TYPES)]
        resources["Res%d%s" % (k, t.split("::")[-1])] = _resource(r, t, k)
    return {"AWSTemplateFormatVersion": "2010-09-09", "Resources": resources}


def cfn_corpus(n, start=0, n_resources=50):
    return [json.dumps(cfn_doc(start + i, n_resources), separators=(",", ":")) for i in range(n)]


IAM_RULES = """
let iam_roles = Resources.*[ Type == 'AWS::IAM::Role' ]

rule IAM_ROLE_NO_WILDCARD_ACTIONS when %iam_roles !empty {
    %iam_roles.Properties.Policies[*].PolicyDocument.Statement[*] {
        when Effect == 'Allow' {
            Action != '*'
            Resource exists
        }
    }
}

rule IAM_ROLE_TRUSTS_SERVICES when %iam_roles !empty {
    %iam_roles.Properties.AssumeRolePolicyDocument.Statement[*].Principal.Service[*] in
        ['ec2.amazonaws.com', 'lambda.amazonaws.com']
}
"""

EBS_RULES = """
rule EBS_VOLUMES_ENCRYPTED {
    AWS::EC2::Volume {
        Properties.Encrypted exists
        Properties.Encrypted == true <<EBS volumes must be encrypted>>
        Properties.Size <= 256
    }
}
"""


# ---------------------------------------------------------------------------------------------
# cfg 4 (BASELINE.json configs[3]): Terraform plan JSON -- planned_values with a
# root module and nested child modules (nesting depth 6-10 under the plan root) and a
# resource_changes array, 200-2000 entries per plan at full size.  Doc i: xorshift32 seed 4242 ^ i.

TF_TYPES = ["aws_s3_bucket", "aws_instance", "aws_iam_role", "aws_security_group", "aws_db_instance"]


def _tf_values(r, t, k):
    if t == "aws_s3_bucket":
        v = {"bucket": "tf-bucket-%d" % k, "acl": r.pick(["private", "public-read", "log-delivery-write"]),
             "force_destroy": r.chance(0.3)}
        if r.chance(0.7):
            v["tags"] = {"Name": "b%d" % k, "Environment": r.pick(["Dev", "Prod", "null"])}
        elif r.chance(0.5):
            v["tags"] = None
        if r.chance(0.6):
            v["versioning"] = [{"enabled": r.chance(0.7), "mfa_delete": False}]
        if r.chance(0.5):
            v["server_side_encryption_configuration"] = [{"rule": [{"apply_server_side_encryption_by_default": [
                {"sse_algorithm": r.pick(["aws:kms", "AES256"]), "kms_master_key_id": None}]}]}]
        return v
    if t == "aws_instance":
        v = {"ami": "ami-%08x" % r.next(), "instance_type": r.pick(["t3.micro", "m5.large", "c5.xlarge", "t2.nano"]),
             "monitoring": r.chance(0.5), "ebs_optimized": r.chance(0.6)}
        if r.chance(0.8):
            v["root_block_device"] = [{"encrypted": r.chance(0.7), "volume_size": 8 + r.next() % 200,
                                       "volume_type": r.pick(["gp2", "gp3"])}]
        if r.chance(0.6):
            v["tags"] = {"Name": "i%d" % k}
        return v
    if t == "aws_iam_role":
        return {"name": "role-%d" % k, "max_session_duration": 3600 * (1 + r.next() % 12),
                "assume_role_policy": json.dumps({"Version": "2012-10-17", "Statement": [
                    {"Effect": "Allow", "Principal": {"Service": r.pick(["ec2.amazonaws.com", "lambda.amazonaws.com"])},
                     "Action": "sts:AssumeRole"}]}, separators=(",", ":"))}
    if t == "aws_security_group":
        ing = []
        for _ in range(1 + r.next() % 3):
            port = r.pick([22, 80, 443, 3389])
            ing.append({"from_port": port, "to_port": port, "protocol": "tcp",
                        "cidr_blocks": [r.pick(["0.0.0.0/0", "10.0.0.0/8", "172.16.0.0/12"])],
                        "description": r.pick(["ssh", "web", "rdp", ""])})
        return {"name": "sg-%d" % k, "ingress": ing, "egress": [{"from_port": 0, "to_port": 0, "protocol": "-1",
                                                                  "cidr_blocks": ["0.0.0.0/0"]}]}
    return {"engine": r.pick(["mysql", "postgres"]), "storage_encrypted": r.chance(0.6),
            "publicly_accessible": r.chance(0.2), "backup_retention_period": r.next() % 14,
            "allocated_storage": 20 + r.next() % 1000}


def _tf_module(r, prefix, n, depth, k0):
    res = []
    for k in range(n):
        t = TF_TYPES[r.next() % len(TF_TYPES)]
        name = "r%d" % (k0 + k)
        res.append({"address": "%s%s.%s" % (prefix, t, name), "mode": "managed", "type": t, "name": name,
                    "provider_name": "registry.terraform.io/hashicorp/aws", "schema_version": 0,
                    "values": _tf_values(r, t, k0 + k)})
    mod = {"resources": res}
    if depth > 0:
        child = _tf_module(r, "%smodule.m%d." % (prefix, depth), max(1, n // 4), depth - 1, k0 + n)
        child["address"] = "%smodule.m%d" % (prefix, depth)
        mod["child_modules"] = [child]
    return mod


def tf_plan_doc(i, n_resources=200):
    r = XorShift32(4242 ^ i)
    depth = 2 + r.next() % 3   # module nesting: the deepest leaf values sit 6-10 levels below the root
    root = _tf_module(r, "", n_resources, depth, 0)
    changes = []
    for res in root["resources"]:
        act = r.pick([["create"], ["update"], ["no-op"], ["delete", "create"]])
        changes.append({"address": res["address"], "mode": "managed", "type": res["type"], "name": res["name"],
                        "change": {"actions": act, "before": None if act == ["create"] else res["values"],
                                   "after": res["values"], "after_unknown": {}}})
    return {"format_version": "1.1", "terraform_version": "1.5.7",
            "planned_values": {"root_module": root}, "resource_changes": changes}


def tf_corpus(n, start=0, n_resources=200):
    return [json.dumps(tf_plan_doc(start + i, n_resources), separators=(",", ":")) for i in range(n)]


def tf_bench_size(i):
    """resources of bench plan i: 200-2000, seeded (xorshift32 seed 9191 ^ i), SURVEY.md 8(d) cfg 4"""
    return 200 + XorShift32(9191 ^ i).next() % 1801


def tf_bench_corpus(n, start=0):
    """the cfg-4 bench corpus: plan i = tf_plan_doc(i, tf_bench_size(i)) (200-2000 resource_changes,
    module nesting putting the deepest values 6-10 levels below the root)"""
    return [json.dumps(tf_plan_doc(start + i, tf_bench_size(start + i)), separators=(",", ":")) for i in range(n)]


# ---------------------------------------------------------------------------------------------
# cfg 5 (BASELINE.json configs[4]): AWS Config configuration items of one account
# snapshot, wrapped into a CloudFormation-shaped `Resources` map keyed by resource id (the
# network-reachability rules query `Resources.*`).  Each snapshot holds Redshift subnet groups,
# subnets, route-table associations, route tables, routes and gateways with `Ref` joins between
# them, plus configuration-item metadata.  Doc i: xorshift32 seed 5151 ^ i.

def config_snapshot_doc(i, n_groups=4):
    r = XorShift32(5151 ^ i)
    res = {}

    def ci(rid, t, props):
        res[rid] = {"Type": t, "Properties": props,
                    "configurationItemStatus": r.pick(["OK", "ResourceDiscovered", "ResourceDeleted"]),
                    "resourceId": rid, "awsRegion": r.pick(["us-east-1", "eu-west-1"]),
                    "tags": {"owner": r.pick(["net", "data", "sec"])}}

    for g in range(n_groups):
        subnets = ["subnet%da%d" % (g, j) for j in range(1 + r.next() % 3)]
        refs = [{"Ref": s} for s in subnets]
        if r.chance(0.3):
            refs.append("subnet-%08x" % r.next())
        ci("rcsg%d" % g, r.pick(["AWS::Redshift::ClusterSubnetGroup", "AWS::Redshift::ClusterSubnetGroup",
                                 "AWS::RDS::DBSubnetGroup"]), {"SubnetIds": refs, "Description": "group %d" % g})
        rt = "rt%d" % g
        ci(rt, "AWS::EC2::RouteTable" if r.chance(0.9) else "AWS::EC2::Subnet", {"VpcId": {"Ref": "vpc"}})
        gw = "gw%d" % g
        ci(gw, r.pick(["AWS::EC2::InternetGateway", "AWS::EC2::TransitGateway", "AWS::EC2::NatGateway"]), {})
        ci("route%d" % g, "AWS::EC2::Route", {"RouteTableId": {"Ref": rt}, "GatewayId": {"Ref": gw},
                                              "DestinationCidrBlock": r.pick(["0.0.0.0/0", "10.0.0.0/8"])})
        for s in subnets:
            ci(s, "AWS::EC2::Subnet" if r.chance(0.95) else "AWS::EC2::Instance",
               {"CidrBlock": "10.%d.%d.0/24" % (g, r.next() % 256), "MapPublicIpOnLaunch": r.chance(0.3),
                "VpcId": {"Ref": "vpc"}})
            ci("assoc-%s" % s, "AWS::EC2::SubnetRouteTableAssociation", {"SubnetId": {"Ref": s},
                                                                          "RouteTableId": {"Ref": rt}})
    ci("vpc", "AWS::EC2::VPC", {"CidrBlock": "10.0.0.0/16", "EnableDnsSupport": True})
    return {"Resources": res}


def config_corpus(n, start=0, n_groups=4):
    return [json.dumps(config_snapshot_doc(start + i, n_groups), separators=(",", ":")) for i in range(n)]


# ---- CloudFormation YAML (block style) -------------------------------------------------------------
# The cfn_doc templates written as YAML the way CloudFormation authors write them: block mappings,
# indented and indentless sequences, compact `- Key: v` entries, flow sequences of scalars, short-form
# intrinsic tags (!Ref, !GetAtt, !Sub, !Join ...), plain / single- / double-quoted scalars and comments,
# with the choices drawn from a XorShift32 per document (deterministic).  The device YAML loader and the
# host libyaml loader must build the same arena from it (tests/test_gpu_yaml.py).

_YAML_INDICATORS = set("-?:,[]{}#&*!|>'\"%@`")
_YAML_WORDS = {"true", "false", "yes", "no", "on", "off", "y", "n", "~", "null", "Null", "NULL", "True", "False",
               "TRUE", "FALSE", "Yes", "No", "YES", "NO", "On", "Off", "ON", "OFF", "Y", "N"}
_FN_SHORT = {"Ref": ("Ref", True, False), "Fn::GetAtt": ("GetAtt", True, True), "Fn::Sub": ("Sub", True, True),
             "Fn::Base64": ("Base64", True, False), "Fn::Join": ("Join", False, True),
             "Fn::Select": ("Select", False, True), "Fn::If": ("If", False, True), "Fn::Equals": ("Equals", False, True),
             "Fn::FindInMap": ("FindInMap", False, True), "Fn::ImportValue": ("ImportValue", True, False)}


def _numeric_like(s):
    t = s[1:] if s[:1] in "+-" else s
    if t.lower() in ("inf", "infinity", "nan"):
        return True
    digits = any(c.isdigit() for c in t)
    return digits and all(c.isdigit() or c in ".eE+-" for c in t)


def _plain_ok(s, flow=False):
    if not s or s != s.strip() or s in _YAML_WORDS or _numeric_like(s):
        return False
    if s[0] in _YAML_INDICATORS or ": " in s or " #" in s or s.endswith(":") or "\n" in s:
        return False
    if any(ord(c) < 0x20 or ord(c) == 0x7F or ord(c) > 0x7E for c in s):
        return False
    if flow and any(c in s for c in ",[]{}:"):
        return False
    return True


def _yaml_scalar(v, rng, flow=False):
    if v is None:
        return "null" if rng.next() % 2 else "~"
    if v is True or v is False:
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return json.dumps(v)
    s = str(v)
    pick = rng.next() % 5
    if _plain_ok(s, flow) and pick < 3:
        return s
    if pick == 3 and "\\" not in s and all(0x20 <= ord(c) < 0x7F for c in s):
        return "'" + s.replace("'", "''") + "'"
    return json.dumps(s, ensure_ascii=False)


def _yaml_key(k, rng):
    return k if _plain_ok(k) and rng.next() % 6 else json.dumps(k, ensure_ascii=False)


def _yaml_fn(v, rng):
    """a short-form tag for a one-key intrinsic function map, or None"""
    if not isinstance(v, dict) or len(v) != 1:
        return None
    (k, x), = v.items()
    if k not in _FN_SHORT or rng.next() % 4 == 0:
        return None
    short, single, seq = _FN_SHORT[k]
    if single and isinstance(x, str) and _plain_ok(x):
        return "!%s %s" % (short, x)
    if seq and isinstance(x, list) and x and all(isinstance(e, (str, int)) and (not isinstance(e, str) or _plain_ok(e, True))
                                                 for e in x):
        return "!%s [%s]" % (short, ", ".join(str(e) for e in x))
    return None


def _yaml_lines(v, indent, rng, out):
    pad = " " * indent
    if isinstance(v, dict):
        for k, x in v.items():
            if rng.next() % 13 == 0:
                out.append(pad + "# " + str(k).lower())
            key = _yaml_key(k, rng)
            fn = _yaml_fn(x, rng)
            if fn is not None:
                out.append("%s%s: %s" % (pad, key, fn))
            elif isinstance(x, dict) and x:
                out.append("%s%s:" % (pad, key))
                _yaml_lines(x, indent + 2, rng, out)
            elif isinstance(x, list) and x:
                if all(not isinstance(e, (dict, list)) for e in x) and rng.next() % 3 == 0 and \
                        all(not isinstance(e, str) or _plain_ok(e, True) for e in x):
                    out.append("%s%s: [%s]" % (pad, key, ", ".join(_yaml_scalar(e, rng, True) for e in x)))
                else:
                    out.append("%s%s:" % (pad, key))
                    _yaml_lines(x, indent + (2 if rng.next() % 2 else 0), rng, out)
            elif isinstance(x, dict):
                out.append("%s%s: {}" % (pad, key))
            elif isinstance(x, list):
                out.append("%s%s: []" % (pad, key))
            else:
                tail = "  # note" if rng.next() % 17 == 0 else ""
                out.append("%s%s: %s%s" % (pad, key, _yaml_scalar(x, rng), tail))
    else:
        for x in v:
            if isinstance(x, dict) and x and _yaml_fn(x, rng) is None:
                sub = []
                _yaml_lines(x, indent + 2, rng, sub)
                out.append(pad + "- " + sub[0][indent + 2:])
                out.extend(sub[1:])
            elif isinstance(x, list) and x:
                out.append(pad + "-")
                _yaml_lines(x, indent + 2, rng, out)
            elif isinstance(x, (dict, list)):
                fn = _yaml_fn(x, rng)
                out.append(pad + "- " + (fn if fn else ("{}" if isinstance(x, dict) else "[]")))
            else:
                out.append(pad + "- " + _yaml_scalar(x, rng))


def cfn_yaml_doc(i, n_resources=50):
    """synthetic template i (cfn_doc's content) as block-style CloudFormation YAML"""
    rng = XorShift32(0x9E3779B9 ^ (i * 2654435761 & 0xFFFFFFFF) or 1)
    out = ["---"] if rng.next() % 3 == 0 else []
    if rng.next() % 2:
        out.append("# synthetic template %d" % i)
    _yaml_lines(cfn_doc(i, n_resources), 0, rng, out)
    return "\n".join(out) + "\n"


def cfn_yaml_corpus(n, start=0, n_resources=50):
    return [cfn_yaml_doc(start + i, n_resources) for i in range(n)]
