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
