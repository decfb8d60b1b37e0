"""Wire contracts built in code (no protoc in the image): the arena ``inference``
package (``inference_api``) and the KServe-v2 predict protocol (``kserve``)."""
