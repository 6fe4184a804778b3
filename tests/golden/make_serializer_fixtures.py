"""Copies the reference's own serializer test data (data files, not source) into
tests/golden/serializer/, run in the build container where /root/reference exists:

* flink-runtime/src/test/resources/stream-element-serializer-<v>/test-data: the 13 bytes
  StreamElementSerializerUpgradeTest (flink-runtime/src/test/java/org/apache/flink/streaming/
  runtime/streamrecord/StreamElementSerializerUpgradeTest.java:63-68) wrote for
  StreamRecord("key", 123456) -- tag 0 (TAG_REC_WITH_TIMESTAMP), the big-endian timestamp,
  then StringSerializer's "key";
* flink-core/src/test/resources/long-serializer-<v>/test-data: the 8 bytes LongSerializer
  wrote for 1234567890L (flink-core/src/test/java/org/apache/flink/api/common/typeutils/base/
  BasicTypeSerializerUpgradeTestSpecifications.java:622,636), big-endian.

Every version directory holds the same bytes (checked here); the newest one is copied, and
serializer/provenance.json records the versions compared."""
import json
import os

REF = "/root/reference"
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "serializer")
SETS = {
    "stream-element-serializer": "flink-runtime/src/test/resources",
    "long-serializer": "flink-core/src/test/resources",
}


def version_key(v):
    return tuple(int(x) for x in v.split("."))


def main():
    os.makedirs(HERE, exist_ok=True)
    prov = {}
    for name, root in SETS.items():
        base = os.path.join(REF, root)
        vers = sorted((d[len(name) + 1:] for d in os.listdir(base) if d.startswith(name + "-")), key=version_key)
        datas = {v: open(os.path.join(base, f"{name}-{v}", "test-data"), "rb").read() for v in vers}
        newest = vers[-1]
        assert all(d == datas[newest] for d in datas.values()), f"{name}: versions differ"
        with open(os.path.join(HERE, f"{name}.test-data"), "wb") as f:
            f.write(datas[newest])
        prov[name] = {"source": f"{root}/{name}-{newest}/test-data", "identical_versions": vers,
                      "hex": datas[newest].hex()}
    with open(os.path.join(HERE, "provenance.json"), "w") as f:
        json.dump(prov, f, indent=1)


if __name__ == "__main__":
    main()
